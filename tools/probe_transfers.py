"""Prints host<->device transfer ceilings (GB/s) measured by the native probe (transfer_probe.hip)."""
import json
import sys

sys.path.insert(0, ".")
from mpi_openmp_cuda_amd import _lib  # noqa: E402

names = ["h2d_memcpy", "d2h_memcpy", "h2d+d2h_concurrent", "zero_copy_read", "zero_copy_write", "d2d_memcpy",
         # the streaming search's 3:1 in/out mix, reported as bytes IN per second
         "mix3to1_zc_read+zc_write", "mix3to1_h2d_memcpy+zc_write", "mix3to1_h2d+d2h_memcpy", "mix3to1_zc_read+d2h_memcpy"]
res = {}
for mb in (16, 256):
    for kind, name in enumerate(names):
        res[f"{name}_{mb}MB"] = round(_lib.lib().moc_transfer_probe(kind, mb << 20, 10 if mb == 16 else 4), 2)
print(json.dumps(res, indent=1))
