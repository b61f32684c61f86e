"""Native RCCL data plane (csrc/comm/rccl_comm.cpp, parallel/rccl.py) on one rank: the weighted all-reduce equals
x * w bitwise, a plain sum leaves x unchanged, the collective captured in a hipGraph replays, and a one-rank
bench-style federation over it aggregates exactly like the ProcessGroup path."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _native():
    from fed_tgan_amd.ops import native
    native.require()
    from fed_tgan_amd.parallel.rccl import NativeRccl
    return NativeRccl(0, 1, DEV)


def test_native_rccl_weighted_all_reduce_one_rank():
    c = _native()
    try:
        x = torch.randn(3_000_001, device=DEV)
        y = x.clone()
        c.all_reduce(y, 0.37)
        torch.cuda.synchronize()
        assert torch.equal(y, x * 0.37)
        z = x.clone()
        c.all_reduce(z, 1.0)
        torch.cuda.synchronize()
        assert torch.equal(z, x)
    finally:
        c.destroy()


def test_native_rccl_all_reduce_captured_in_a_graph():
    c = _native()
    try:
        buf = torch.zeros(1 << 20, device=DEV)
        s = torch.cuda.Stream(DEV)
        s.wait_stream(torch.cuda.current_stream(DEV))
        with torch.cuda.stream(s):          # warm-up outside the capture
            c.all_reduce(buf, 0.5)
        torch.cuda.current_stream(DEV).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            buf.mul_(2.0)
            c.all_reduce(buf, 0.5)          # weight baked into the graph
        src = torch.randn(1 << 20, device=DEV)
        for _ in range(3):
            buf.copy_(src)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(buf, (src * 2.0) * 0.5)
    finally:
        c.destroy()


def test_native_rccl_plane_in_a_one_rank_federation(tmp_path):
    """Comm(native_rccl=True) over a one-rank process group: the round's all-reduce goes through the native
    communicator and the trained model equals the ProcessGroup path's bitwise."""
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.parallel.comm import Comm
    flats = []
    for native_plane in (False, True):
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        comm = Comm(0, 1, [0], "nccl", port=port, device=DEV, force_dist=True, native_rccl=native_plane)
        try:
            assert (comm._native is not None) == native_plane
            cfg = FedConfig(spec=intrusion_spec(), epochs=2, synthetic_rows=4000, out_dir=str(tmp_path / str(native_plane)),
                            backend="hip", gmm_backend="torch", verbose=False)
            rt = FedRuntime(cfg, comm, DEV)
            rt.initialize()
            rt.fit()
            torch.cuda.synchronize()
            flats.append(rt.engine.flat.clone())
        finally:
            comm.destroy()
    assert torch.equal(flats[0], flats[1])
