"""mCGC benchmark model (reference: scripts/benchmark_models/cgc_modified.py) -> gnn.cgc."""
from gnn.cgc import CGCLayer, CrystGraphConv  # noqa: F401
