"""Import-path twin of the reference's ``scripts/benchmark_models`` package, so the
reference training scripts' ``from benchmark_models.cgc_modified import CrystGraphConv``
resolves to the HIP implementations in ``gnn.cgc``."""
