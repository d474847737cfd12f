"""I/O, CLI, timers and logging helpers."""
