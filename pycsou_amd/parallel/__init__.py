"""Multi-GPU execution of the fused PDS loop: row slabs, one process per GPU."""

from .slab import DistComm, SlabLayout, SlabPDS2D, gather_rows, row_split, run_local, run_local_deep  # noqa: F401
