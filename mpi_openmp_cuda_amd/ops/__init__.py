"""Search ops (CPU OpenMP engine, gfx950 HIP engine)."""
