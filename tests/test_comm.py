"""The data-plane choice is agreed by every rank (Comm._vote_data_backend): ranks whose local
view differs -- a CPU-only dedicated federator next to a GPU client, or two clients on one device -- must
not end up in different process groups (that hung init until the process-group timeout)."""
import torch
import torch.multiprocessing as mp

from fed_tgan_amd.cli import free_port
from fed_tgan_amd.parallel.comm import Comm

# (rank devices, client ranks, auto mode) -> the backend every rank must agree on
CASES = [
    (["cpu", "cuda:0"], [0, 1], "auto", "gloo"),          # colocated, one rank without a GPU
    (["cuda:0", "cuda:0"], [0, 1], "auto", "gloo"),       # two clients on one device (RCCL: one rank per GPU)
    (["cpu", "cpu"], [1], "auto", "gloo"),
    (["cpu", "cuda:0"], [1], "auto_all", "gloo"),         # MD-GAN: the federator joins the P2P group too
]


def _worker(rank, port, devs, clients, mode, out):
    # the vote reads device identities only; nothing is allocated on the (possibly absent) GPU
    comm = Comm.__new__(Comm)
    comm.rank, comm.world_size, comm.client_ranks = rank, len(devs), list(clients)
    comm.device = torch.device(devs[rank])
    import datetime
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=len(devs),
                            timeout=datetime.timedelta(seconds=60))
    comm.ctrl = dist.group.WORLD
    out[rank] = comm._vote_data_backend(mode == "auto_all")
    dist.destroy_process_group()


def test_data_backend_vote_agrees():
    for devs, clients, mode, want in CASES:
        out = mp.Manager().dict()
        mp.spawn(_worker, args=(free_port(), devs, clients, mode, out), nprocs=len(devs), join=True)
        assert [out[r] for r in range(len(devs))] == [want] * len(devs), (devs, clients, mode, dict(out))


def test_pick_data_backend():
    """RCCL only when every member rank has its own (host, device)."""
    pick = Comm.pick_data_backend
    assert pick([(True, "cuda", "h", i) for i in range(4)] + [(False, "cpu", "h", -1)]) == "nccl"
    assert pick([(True, "cuda", "h", 0), (True, "cuda", "h2", 0)]) == "nccl"       # two hosts, device 0 each
    assert pick([(True, "cuda", "h", 0), (True, "cuda", "h", 0)]) == "gloo"
    assert pick([(True, "cuda", "h", 0), (True, "cpu", "h", -1)]) == "gloo"
    assert pick([(False, "cuda", "h", 0)]) == "gloo"


def _share_worker(rank, port, out):
    """Dedicated federator (rank 0) + two clients with an "RCCL" data plane, emulated on gloo: the hand-off of
    the aggregate goes first client -> federator over the pair group; the second client takes no part."""
    import datetime
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=3,
                            timeout=datetime.timedelta(seconds=60))
    comm = Comm.__new__(Comm)
    comm.rank, comm.world_size, comm.client_ranks = rank, 3, [1, 2]
    comm.device = torch.device("cpu")
    comm.data_backend, comm.dist_active, comm._share = "nccl", True, None
    comm.ctrl = dist.group.WORLD
    comm.share_pg = {0: dist.new_group(ranks=[0, 1], backend="gloo")}
    flat = torch.full((64,), float(rank))
    extra = torch.full((4,), 10.0 + rank) if rank else torch.zeros(4)
    res = []
    for rnd in range(3):      # several rounds: a rank that skipped a collective would pair it with the next one
        shared = comm.share_with_federator(flat, 0, extra=extra)
        res.append(bool(shared))
        # the runtime's follow-up (FedRuntime._sync_losses): a control all-reduce only when NOT shared -- it must
        # be skipped (or taken) by every rank alike
        if not shared:
            dist.all_reduce(torch.zeros(1), group=comm.ctrl)
        dist.barrier(group=comm.ctrl)
    if rank == 1:
        comm._share[3].result()
    out[rank] = (res, flat[0].item(), extra[0].item())
    dist.destroy_process_group()


def test_share_with_federator_is_collective():
    """with a dedicated federator and >= 2 clients, share_with_federator returned True on the
    first client and the federator only, so the other clients ran a control all-reduce the first two skipped
    (a deadlock, or a mis-paired collective the next round)."""
    out = mp.Manager().dict()
    mp.spawn(_share_worker, args=(free_port(), out), nprocs=3, join=True)
    assert [out[r][0] for r in range(3)] == [[True] * 3] * 3, dict(out)
    assert out[0][1] == 1.0 and out[0][2] == 11.0       # the federator received the first client's aggregate
