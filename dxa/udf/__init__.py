"""User extension points: scalar UDFs, dynamic (stateful, per-batch refreshed) UDFs, UDAFs, HTTP ("Azure Function")
UDFs, raw-string normalizers and pre-projection hooks.  See ``dxa.udf.api`` for the plugin contracts."""
