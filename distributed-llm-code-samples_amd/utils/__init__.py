"""Config, data, checkpointing, metrics, profiling."""
