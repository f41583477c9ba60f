"""MI355X-native EnergyEquivGNN hot path (drop-in for the reference ``gnn`` package).

``from gnn import EnergyEquivGNN`` works as in ``scripts/train_main.py:21`` once
``energy-equiv-lattice-gnn_amd/`` is on ``sys.path``.  ``GLAMM_Dataset`` builds the
reference's graphs from catalogue entries (``gnn.lattice_data``); reading ``.lat`` files
themselves needs the un-vendored ``lattices`` package and raises.
"""
from .model import EnergyEquivGNN, GNN_Head  # noqa: F401
from .synthetic import SyntheticLattices, make_lattice  # noqa: F401
from .data import Batch, Data, DataLoader, collate  # noqa: F401
from .train import LightningWrappedModel, stiffness_loss  # noqa: F401
from .lattice_data import GLAMM_Dataset, RotateLat, process_lattice  # noqa: F401

__all__ = ["GLAMM_Dataset", "EnergyEquivGNN"]
classes = __all__
