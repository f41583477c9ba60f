"""MI355X-native EnergyEquivGNN hot path (drop-in for the reference ``gnn`` package).

``from gnn import EnergyEquivGNN`` works as in ``scripts/train_main.py:21`` once
``energy-equiv-lattice-gnn_amd/`` is on ``sys.path``.  ``GLAMM_Dataset`` (the
``.lat`` catalogue reader) is out of scope for this round; the
name is exported and raises with a pointer to the synthetic generator.
"""
from .model import EnergyEquivGNN, GNN_Head  # noqa: F401
from .synthetic import SyntheticLattices, make_lattice  # noqa: F401
from .data import Batch, Data, DataLoader, collate  # noqa: F401
from .train import LightningWrappedModel, stiffness_loss  # noqa: F401


class GLAMM_Dataset:  # noqa: N801
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            "GLAMM_Dataset needs the external GLAMM catalogue and the 'lattices' submodule "
            "(gnn/datasets.py:25-307); use gnn.SyntheticLattices for benchmarking")


__all__ = ["GLAMM_Dataset", "EnergyEquivGNN"]
classes = __all__
