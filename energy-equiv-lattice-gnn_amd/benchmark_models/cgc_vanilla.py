"""CGC benchmark model (reference: scripts/benchmark_models/cgc_vanilla.py) -> gnn.cgc."""
from gnn.cgc import CGCLayer  # noqa: F401
from gnn.cgc import CrystGraphConvVanilla as CrystGraphConv  # noqa: F401
