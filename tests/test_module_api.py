"""CPU: the drop-in modules mirror the reference's constructor, module tree and state_dict keys
(notorch/nn/gnn/chemprop.py:49-75, residual.py:21-28, agg.py:15-47), and refuse CPU tensors
(the product has no CPU fallback)."""
import pytest
import torch
import torch.nn as nn

from notorch_amd.data.models.graph import BatchedGraph, Graph
from notorch_amd.nn import ChempropBlock, ChempropLayer, Max, Mean, Residual, Sum


def test_state_dict_keys_residual():
    blk = ChempropBlock(hidden_dim=32, depth=3)
    keys = list(blk.state_dict())
    assert keys == [
        f"layers.{i}.module.update.0.{p}" for i in range(3) for p in ("weight", "bias")
    ]
    assert all(isinstance(m, Residual) for m in blk.layers)
    assert blk.depth == 3 and blk.hidden_dim == 32 and blk.reduce == "sum"


def test_state_dict_keys_no_residual_no_bias():
    blk = ChempropBlock(hidden_dim=16, depth=2, residual=False, bias=False)
    assert list(blk.state_dict()) == ["layers.0.update.0.weight", "layers.1.update.0.weight"]


def test_shared_layers_are_one_module():
    blk = ChempropBlock(hidden_dim=16, depth=3, shared=True)
    inner = [m.module for m in blk.layers]
    assert inner[0] is inner[1] is inner[2]
    # state_dict repeats the shared tensor under every index (chemprop.py:65-66)
    sd = blk.state_dict()
    assert len(sd) == 6
    assert sd["layers.0.module.update.0.weight"].data_ptr() == sd["layers.2.module.update.0.weight"].data_ptr()
    assert len(list(blk.parameters())) == 2


def test_reference_state_dict_loads():
    """A state_dict saved from a reference-shaped module loads unchanged (same keys/shapes)."""
    blk = ChempropBlock(hidden_dim=24, depth=2)
    sd = {k: torch.randn_like(v) for k, v in blk.state_dict().items()}
    blk2 = ChempropBlock(hidden_dim=24, depth=2)
    blk2.load_state_dict(sd)
    assert torch.equal(blk2.layers[1].module.update[0].weight, sd["layers.1.module.update.0.weight"])


def test_layer_repr_and_defaults():
    layer = ChempropLayer(8)
    assert "(reduce): sum" in repr(layer)
    assert isinstance(layer.act, nn.ReLU) and isinstance(layer.update[1], nn.Dropout)
    with pytest.raises(ValueError):
        ChempropLayer(8, reduce="median")


def _tiny_graph():
    Xv = torch.randn(3, 4)
    Xe = torch.randn(4, 4)
    ei = torch.tensor([[0, 1, 1, 2], [1, 0, 2, 1]])
    return Xv, Xe, ei, torch.tensor([1, 0, 3, 2])


def test_cpu_tensors_raise_no_fallback():
    Xv, Xe, ei, rev = _tiny_graph()
    with pytest.raises(RuntimeError, match="ROCm"):
        ChempropBlock(4, depth=1)(Graph(Xv, Xe, ei, rev))
    BG = BatchedGraph(Xv, Xe, ei, rev, batch_node_index=torch.zeros(3, dtype=torch.long),
                      batch_edge_index=torch.zeros(4, dtype=torch.long), size=1)
    for R in (Sum, Mean, Max):
        with pytest.raises(RuntimeError, match="ROCm"):
            R()(BG)


def test_unsupported_activation_rejected():
    from notorch_amd import kernels

    with pytest.raises(NotImplementedError):
        kernels.act_code(nn.Softplus())
    assert kernels.act_code(nn.LeakyReLU(0.2))[1] == pytest.approx(0.2)


def test_graph_update_is_shallow_copy():
    Xv, Xe, ei, rev = _tiny_graph()
    G = Graph(Xv, Xe, ei, rev)
    G2 = G.update(node_feats=torch.zeros(3, 4))
    assert G2 is not G and G2.edge_index is G.edge_index and torch.equal(G.node_feats, Xv)
    assert G.update(in_place=True, edge_feats=Xe) is G
    assert G.num_nodes == 3 and G.num_edges == 4
    assert G.dense2sparse[1, 2] == 2 and G.A.sum() == 4


def test_mlp_head_module_tree_matches_reference_layout():
    """MLP (reference nn/mlp.py:9-68): Linear, act, Dropout, ..., Linear (+ Unflatten), so state_dict keys
    and the output shape are the reference's; default hidden_dim 256 (notorch/conf.py:11)."""
    import torch.nn as nn

    from notorch_amd.nn import MLP

    m = MLP(300, 1)
    assert [type(x) for x in m] == [nn.Linear, nn.ReLU, nn.Dropout, nn.Linear]
    assert list(m.state_dict()) == ["0.weight", "0.bias", "3.weight", "3.bias"]
    assert m[0].out_features == 256 and m[3].out_features == 1
    m = MLP(300, (2, 3), hidden_dim=64, num_layers=2, dropout=0.1, activation=nn.SiLU)
    assert [type(x) for x in m] == [nn.Linear, nn.SiLU, nn.Dropout, nn.Linear, nn.SiLU, nn.Dropout, nn.Linear,
                                    nn.Unflatten]
    assert m[2].p == 0.1 and m[6].out_features == 6
    assert m(torch.randn(5, 300)).shape == (5, 2, 3)
    m = MLP(300, 5, num_layers=0)
    assert [type(x) for x in m] == [nn.Linear] and m[0].in_features == 300 and m[0].out_features == 5
