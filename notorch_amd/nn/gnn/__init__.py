from notorch_amd.nn.gnn.agg import Aggregation, Gated, Max, Mean, Min, SDPAttention, Sum
from notorch_amd.nn.gnn.chemprop import ChempropBlock, ChempropLayer
from notorch_amd.nn.gnn.embed import EmbeddedChempropBlock, GraphEmbedding

__all__ = ["Aggregation", "Gated", "SDPAttention", "Max", "Mean", "Min", "Sum", "ChempropBlock", "ChempropLayer", "GraphEmbedding",
           "EmbeddedChempropBlock"]
