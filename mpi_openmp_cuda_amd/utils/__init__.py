"""I/O, synthetic data, timers."""
