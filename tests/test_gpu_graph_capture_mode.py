"""The HIP runtime's graph capture mode (mapf_amd/__init__.py).  With ROCm 7's packet
capture (DEBUG_CLR_GRAPH_PACKET_CAPTURE=1, the runtime default) a captured hipMemsetAsync takes
effect on the first replay only, so captured multi-block torch reductions -- their semaphores are
zeroed by a captured memset -- return stale partial sums from the second replay on
(profiles/r05_diag20_packet_capture_{on,off}.log).  mapf_amd (and tests/conftest.py) switch the mode off before the runtime
starts; these tests pin that the replays are then right, including the autocast Linear whose
captured bias gradient went wrong, and that Model falls back to an eager update when a process runs
with the mode on."""
import ctypes
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")


def _capture(fn):
    g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out = fn()
    torch.cuda.current_stream().wait_stream(s)
    return g, out


def test_capture_mode_is_off_in_this_process():
    import mapf_amd
    assert os.environ.get(mapf_amd.GRAPH_CAPTURE_FLAG) == "0"


@pytest.mark.parametrize("shape,dim", [((1088, 1536), 0), ((8192, 1536), 0), ((1088, 1536), None),
                                       ((64, 1536), 0), ((1088, 1536), 1)])
def test_captured_reductions_replay_right(shape, dim):
    _need_gpu()
    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda")
    fn = (lambda: x.sum().reshape(1)) if dim is None else (lambda: x.sum(dim))
    want = fn()
    g, y = _capture(fn)
    for _ in range(4):
        y.fill_(float("nan"))                 # an output the replay does not write shows up
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(y, want, rtol=1e-5, atol=1e-4)


def test_captured_memset_replays():
    _need_gpu()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    buf = torch.zeros(64, dtype=torch.int32, device="cuda")
    rc = []

    def body():
        rc.append(hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, buf.numel() * 4,
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        buf.add_(1)
    g, _ = _capture(body)
    assert rc == [0]
    for _ in range(4):
        buf.fill_(7)
        g.replay()
        torch.cuda.synchronize()
        assert torch.all(buf == 1), buf[:4].tolist()


def test_captured_autocast_linear_bias_grad_after_churn():
    """round 4's failing case: nn.Linear under fp16 autocast, forward + backward
    captured; small NaN tensors allocated and freed between replays; the bias gradient (a captured
    column sum) must equal the eager backward's on every replay."""
    _need_gpu()
    torch.manual_seed(0)
    lin = torch.nn.Linear(512, 1536).cuda()
    x = torch.randn(1088, 512, device="cuda")

    def body():
        lin.weight.grad = lin.bias.grad = None
        with torch.autocast(device_type="cuda", cache_enabled=False):
            y = lin(x)
        (y.float().pow(2).mean() * 256.0).backward()
        return lin.bias.grad, lin.weight.grad
    for _ in range(2):
        want_b, want_w = (t.clone() for t in body())
    g, (gb, gw) = _capture(body)
    for _ in range(5):
        ts = [torch.full((1 << (k % 17),), float("nan"), device="cuda") for k in range(600)]
        torch.cuda.synchronize()
        del ts
        g.replay()
        torch.cuda.synchronize()
        assert torch.isfinite(gb).all()
        torch.testing.assert_close(gb, want_b, rtol=1e-3, atol=1e-3)
        torch.testing.assert_close(gw, want_w, rtol=1e-3, atol=1e-3)


def test_model_update_falls_back_to_eager_under_packet_capture():
    """A process that starts the runtime with the mode ON: captured_reductions_ok sees the stale sums
    and Model.train runs its updates eagerly (finite, no graph)."""
    _need_gpu()
    code = r'''
import os, sys, warnings
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "primal-ppo_amd"), os.path.join(sys.argv[1], "tests")]
import numpy as np, torch
from mapf_amd.model import Model, captured_reductions_ok
from test_gpu_update_graph import _batch
assert os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] == "1"
torch.manual_seed(0)
m = Model(0, "cuda", global_model=True, numChannel=6, num_agents=8, fov=9)
m.net_scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 8)
g = torch.Generator(device="cuda").manual_seed(1)
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    for _ in range(4):
        s = m.train(*_batch(g)[:8], None, _batch(g)[8], 1.0)
        assert all(np.isfinite(float(x)) for x in s), s
upd = next(iter(m._updates.values()))
print("reductions_ok", captured_reductions_ok("cuda"), "graph", upd.graph is not None,
      "eager_runs", upd.eager_runs, "warned", any("eagerly" in str(x.message) for x in w))
'''
    env = dict(os.environ, DEBUG_CLR_GRAPH_PACKET_CAPTURE="1")
    r = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = r.stdout.strip().splitlines()[-1]
    print(line)
    # the runtime may someday replay memsets right in this mode: then the graph is legitimately used
    if "reductions_ok False" in line:
        assert line.endswith("graph False eager_runs 4 warned True"), line
    else:
        assert "graph True" in line, line
