from notorch_amd.nn.gnn.agg import Aggregation, Max, Mean, Min, Sum
from notorch_amd.nn.gnn.chemprop import ChempropBlock, ChempropLayer
from notorch_amd.nn.gnn.embed import EmbeddedChempropBlock, GraphEmbedding

__all__ = ["Aggregation", "Max", "Mean", "Min", "Sum", "ChempropBlock", "ChempropLayer", "GraphEmbedding",
           "EmbeddedChempropBlock"]
