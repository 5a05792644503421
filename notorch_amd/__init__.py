"""notorch_amd — MI355X-native bond-message D-MPNN engine (drop-in for notorch's ChempropBlock path).

Public surface mirrors the reference module paths:
  notorch.nn.gnn.chemprop  -> notorch_amd.nn.gnn.chemprop   (ChempropLayer, ChempropBlock)
  notorch.nn.gnn.agg       -> notorch_amd.nn.gnn.agg        (Aggregation, Sum, Mean, Max)
  notorch.nn.residual      -> notorch_amd.nn.residual       (Residual)
  notorch.data.models.graph-> notorch_amd.data.models.graph (Graph, BatchedGraph + CSR layout)
Kernels: notorch_amd/csrc (HIP, gfx950) behind the C ABI in include/notorch_amd.h.
"""
__version__ = "0.1.0"
