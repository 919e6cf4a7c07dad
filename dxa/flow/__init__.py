"""Control-plane configuration: Flow JSON (the designer's document) → runtime job config (``datax.job.*`` .conf +
transform / projection / schema files).  Reference: Services/DataX.Config/DataX.Config (RuntimeConfigGeneration,
S100…S900 processors, flattener, token templating)."""
