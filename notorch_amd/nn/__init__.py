from notorch_amd.nn.gnn import (
    Aggregation,
    ChempropBlock,
    ChempropLayer,
    EmbeddedChempropBlock,
    GraphEmbedding,
    Max,
    Mean,
    Min,
    Sum,
)
from notorch_amd.nn.residual import Residual

__all__ = [
    "Aggregation", "ChempropBlock", "ChempropLayer", "GraphEmbedding", "EmbeddedChempropBlock", "Max", "Mean", "Min", "Sum", "Residual",
]
