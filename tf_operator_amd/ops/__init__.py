"""Fused gfx950 HIP ops (ctypes-bound, run on torch's current HIP stream)."""
