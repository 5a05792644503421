from notorch_amd.nn.gnn import (
    Aggregation,
    ChempropBlock,
    ChempropLayer,
    EmbeddedChempropBlock,
    Gated,
    GraphEmbedding,
    SDPAttention,
    Max,
    Mean,
    Min,
    Sum,
)
from notorch_amd.nn.mlp import MLP
from notorch_amd.nn.residual import Residual

__all__ = [
    "Aggregation", "Gated", "SDPAttention", "ChempropBlock", "ChempropLayer", "GraphEmbedding", "EmbeddedChempropBlock", "Max", "Mean", "Min", "Sum", "Residual", "MLP",
]
