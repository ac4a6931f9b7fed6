"""Benchmarks of the BASELINE.json headline (see :mod:`.flagship`)."""
