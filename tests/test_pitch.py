"""Row-pitch rule of the inference forward's intermediate H_l / S_l (host logic, no GPU)."""
import torch

from notorch_amd.nn.gnn import _engine


def test_row_pitch_by_graph_size(monkeypatch):
    monkeypatch.setattr(_engine, "_ROW_PAD", True)
    monkeypatch.setattr(_engine, "_ROW_ALIGN", 0)
    big = True  # a hub graph
    assert _engine.row_pitch(300, torch.float32) == 304  # 32-byte sectors
    assert _engine.row_pitch(300, torch.float32, big) == 320  # whole 128-byte L2 lines on hub graphs
    assert _engine.row_pitch(256, torch.float32, big) is None  # already whole lines
    assert _engine.row_pitch(264, torch.float32) is None  # already whole sectors
    assert _engine.row_pitch(264, torch.float32, big) == 288
    assert _engine.row_pitch(300, torch.bfloat16, big) is None  # fp32 only
    assert _engine.row_pitch(100, torch.float32, big) is None  # h < 128
    assert _engine.row_pitch(302, torch.float32, big) is None  # h % 4 != 0
    monkeypatch.setattr(_engine, "_ROW_PAD", False)
    assert _engine.row_pitch(300, torch.float32, big) is None
