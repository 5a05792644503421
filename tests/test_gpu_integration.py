"""GPU integration in the reference's own model pattern (lightning_models/model.py:159-241), mirroring
its regression tests (tests/integration/test_regression.py:50-93).

tensordict / lightning are absent here, so `_TDModule` / `_TDSequential` emulate exactly the call
pattern NotorchModel relies on: ``module(*[td[k] for k in in_keys])`` with the outputs stored
under ``f"{name}.{key}"`` (model.py:159-166, 212, 221-222).  The pipeline is the reference's
encoder: GraphEmbedding -> ChempropBlock -> Sum readout -> MLP head, all notorch_amd modules except
the plain torch head.
* ``test_quick``: one training step runs and every parameter receives a finite gradient
  (``fast_dev_run``, test_regression.py:50-64);
* ``test_overfit``: 100 molecules in batches of 20, 100 epochs, normalised targets, MSE <= 1e-3
  (test_regression.py:67-93), trained through the kernel backward.
"""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

DEV = "cuda"


class _TDModule:
    def __init__(self, name, module, in_keys, out_keys):
        self.name, self.module, self.in_keys, self.out_keys = name, module, in_keys, out_keys

    def __call__(self, td):
        out = self.module(*[td[k] for k in self.in_keys])
        outs = out if isinstance(out, tuple) else (out,)
        for k, v in zip(self.out_keys, outs):
            td[f"{self.name}.{k}"] = v
        return td


class _TDSequential:
    def __init__(self, *mods):
        self.mods = mods

    def __call__(self, td):
        for m in self.mods:
            td = m(td)
        return td


def _model(h=96, depth=3):
    from notorch_amd.nn import ChempropBlock, GraphEmbedding, Sum

    torch.manual_seed(0)
    embed = GraphEmbedding(42, 13, h)
    block = ChempropBlock(hidden_dim=h, depth=depth)
    agg = Sum()
    head = nn.Sequential(nn.Linear(h, h), nn.ReLU(), nn.Linear(h, 1))
    mods = nn.ModuleList([embed, block, agg, head]).to(DEV)
    seq = _TDSequential(
        _TDModule("embed", embed, ["G"], ["G"]),
        _TDModule("encoder", block, ["embed.G"], ["G"]),
        _TDModule("agg", agg, ["encoder.G"], ["X"]),
        _TDModule("head", head, ["agg.X"], ["y"]),
    )
    return mods, seq


def _batches(n=100, bs=20, seed=0):
    from notorch_amd.data.models.graph import BatchedGraph
    from notorch_amd.data.synth import make_batch

    Gs = make_batch("qm9", n, seed=seed).to_graphs()
    g = torch.Generator().manual_seed(seed)
    y = torch.randn(n, 1, generator=g)
    y = (y - y.mean()) / y.std()  # dset.normalize_targets()
    return [(BatchedGraph.from_graphs(Gs[i:i + bs]).to(DEV), y[i:i + bs].to(DEV)) for i in range(0, n, bs)]


def test_quick():
    mods, seq = _model()
    opt = torch.optim.Adam(mods.parameters(), lr=1e-3)
    G, y = _batches()[0]
    td = seq({"G": G})
    loss = (td["head.y"] - y).square().mean()
    loss.backward()
    for name, p in mods.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), name
    opt.step()


def test_overfit():
    mods, seq = _model()
    opt = torch.optim.Adam(mods.parameters(), lr=1e-3)
    data = _batches()
    for _ in range(100):
        for G, y in data:
            opt.zero_grad(set_to_none=True)
            loss = (seq({"G": G})["head.y"] - y).square().mean()
            loss.backward()
            opt.step()
    with torch.no_grad():
        errors = torch.cat([seq({"G": G})["head.y"] - y for G, y in data])
    mse = errors.square().mean().item()
    assert mse <= 1e-3, mse
