"""Control plane: REST services (flow management, jobs, LiveQuery kernels, schema inference, metrics), design-time
storage, the local job manager, the SimulatedData generator service and the metrics ingestor."""
