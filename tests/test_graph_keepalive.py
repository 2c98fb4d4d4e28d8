"""Per-capture workspaces live as long as their graph (VERDICT r03 "what's weak" 9: ops kept every captured
call's workspace in a module list forever, so a process rebuilding step objects grew without bound)."""
import gc

import pytest
import torch


@pytest.mark.gpu
def test_captured_workspace_freed_with_its_graph():
    from adaptive_city_nerf_amd import _lib, ops
    dev = torch.device("cuda")
    pred = torch.rand(4096, 3, device=dev)
    gt = torch.rand(4096, 3, device=dev)
    ops.mse_linear_fwd(pred, gt)          # eager: the per-stream workspace
    torch.cuda.synchronize()
    untracked = len(_lib._UNTRACKED_CAPTURE)
    graphs = []
    for _ in range(3):
        g = torch.cuda.CUDAGraph()
        with _lib.graph_capture(g):
            out = ops.mse_linear_fwd(pred, gt)
        g.replay()
        torch.cuda.synchronize()
        assert len(g._acn_keepalive) >= 1       # the captured call's own workspace rides on the graph
        graphs.append((g, out))
    assert len(_lib._UNTRACKED_CAPTURE) == untracked
    ref = ops.mse_linear_fwd(pred, gt)
    for g, out in graphs:
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    import weakref
    w = weakref.ref(graphs[0][0]._acn_keepalive[0])
    del graphs, g, out
    gc.collect()
    assert w() is None                          # freed with its graph


def test_capture_keepalive_outside_capture_falls_back():
    from adaptive_city_nerf_amd import _lib
    n = len(_lib._UNTRACKED_CAPTURE)
    t = torch.zeros(4)
    assert _lib.capture_keepalive(t) is t
    assert len(_lib._UNTRACKED_CAPTURE) == n + 1
    _lib._UNTRACKED_CAPTURE.pop()
