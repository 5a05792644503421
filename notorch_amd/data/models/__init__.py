from notorch_amd.data.models.graph import BatchedGraph, DeviceLayout, Graph

__all__ = ["BatchedGraph", "DeviceLayout", "Graph"]
