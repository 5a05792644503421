from notorch_amd.data.models.graph import BatchedGraph, Graph

__all__ = ["BatchedGraph", "Graph"]
