"""xGMI IPC collectives (csrc/kernels/ipc_comm.hip) on ONE MI355X: 2 and 3 processes share cuda:0,
exchange HIP IPC handles over a gloo group and all-reduce through each other's mapped buffers.
Checked against the fp32 sum computed on the host from every rank's (seeded) input. On a one-GPU
box the peer reads stay on-device; the same kernels read over xGMI on an 8-GPU node."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASES = [  # (numel, dtype, two_shot_bytes)
    (4, torch.float32, None), (1, torch.float32, None), (1000, torch.bfloat16, None),
    (65536 + 8, torch.float32, None), (300_001, torch.bfloat16, None),
    (262_144, torch.float32, 0),  # forced two-shot
    (1_000_003, torch.bfloat16, 0),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inp(rank, i, n, dtype):
    g = torch.Generator().manual_seed(1000 * i + rank)
    return torch.randn(n, generator=g).to(dtype)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        from gke_ray_train_amd.parallel.ipc import IpcCommunicator
        comms = {None: IpcCommunicator(max_bytes=8 << 20, timeout_s=20.0),
                 0: IpcCommunicator(max_bytes=8 << 20, timeout_s=20.0, two_shot_bytes=0)}
        for i, (n, dt, ts) in enumerate(CASES):
            c = comms[ts]
            t = _inp(rank, i, n, dt).cuda()
            for rep in range(3):  # repeated calls exercise both staging parities
                x = t.clone()
                c.all_reduce(x, average=(rep == 2))
            out[i] = x.float().cpu().numpy()  # by value: a shared-fd tensor dies with this process
        c = comms[None]
        c.barrier()
        torch.cuda.synchronize()
        for c in comms.values():
            c.check()
        # latency: 64 back-to-back 4-byte all-reduces
        x = torch.ones(4, device="cuda")
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        comms[None].barrier()
        ev0.record()
        for _ in range(64):
            comms[None].all_reduce(x)
        ev1.record()
        torch.cuda.synchronize()
        comms[None].check()
        out["us"] = ev0.elapsed_time(ev1) * 1000 / 64
        for c in comms.values():
            c.close()
        q.put((rank, out))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: the full node's rank count (kIpcMaxRanks), peers on one card
def test_ipc_allreduce_matches_host_sum(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, o = q.get(timeout=240)
            res[r] = o
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert isinstance(res[r], dict), f"rank {r}: {res[r]}"
    for i, (n, dt, _ts) in enumerate(CASES):
        exp = sum(_inp(r, i, n, dt).float() for r in range(world)) / world
        tol = 1e-6 if dt == torch.float32 else 1e-2
        for r in range(world):
            got = torch.from_numpy(res[r][i])
            assert torch.allclose(got, exp, atol=tol * 4, rtol=tol), (world, i, r, (got - exp).abs().max())
        for r in range(1, world):  # fixed reduction order: bit-identical on every rank
            assert torch.equal(torch.from_numpy(res[r][i]), torch.from_numpy(res[0][i]))
    print(f"world {world}: 4-byte all-reduce {res[0]['us']:.1f} us")


# ----------------------------------------------------------------------------- buffer shapes
def _shapes_worker(rank, world, port, q):
    """Separately allocated inputs of many sizes (1 element .. exactly the buffer capacity), at
    16-B aligned and unaligned offsets, alternating between two communicators (own buffers and
    epoch sequences, different capacities) so both parities of each are reused many times."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        from gke_ray_train_amd.parallel.ipc import IpcCommunicator
        small = IpcCommunicator(max_bytes=4096, timeout_s=20.0)
        big = IpcCommunicator(max_bytes=1 << 20, timeout_s=20.0, two_shot_bytes=64 << 10)
        cases = []
        for cap_c, c in ((4096, small), (1 << 20, big)):
            for dt in (torch.float32, torch.bfloat16):
                e = torch.tensor([], dtype=dt).element_size()
                for n in (1, 3, 7, 8, 9, cap_c // e - 1, cap_c // e):
                    cases.append((c, n, dt))
        for i, (c, n, dt) in enumerate(cases):
            g = torch.Generator().manual_seed(7000 + 100 * i + rank)
            host = torch.randn(n + 1, generator=g).to(dt)
            buf = host.cuda()                        # its own allocation
            x = buf[1:] if i % 2 else buf[:n]         # odd cases: a view at a 2/4-byte offset
            c.all_reduce(x)
            out[i] = x.float().cpu().numpy()
        try:  # one element beyond the capacity is refused, not truncated
            small.all_reduce(torch.zeros(4096 // 4 + 1, device="cuda"))
            out["over"] = "accepted"
        except ValueError:
            out["over"] = "refused"
        torch.cuda.synchronize()
        small.check()
        big.check()
        small.close()
        big.close()
        q.put((rank, out))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _shape_cases():
    cases = []
    for cap_c in (4096, 1 << 20):
        for dt in (torch.float32, torch.bfloat16):
            e = torch.tensor([], dtype=dt).element_size()
            for n in (1, 3, 7, 8, 9, cap_c // e - 1, cap_c // e):
                cases.append((n, dt))
    return cases


def _spawn(target, world, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, o = q.get(timeout=timeout)
            res[r] = o
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert isinstance(res[r], dict), f"rank {r}: {res[r]}"
    return res


def test_ipc_buffer_sizes_offsets_parities():
    world = 2
    res = _spawn(_shapes_worker, world)
    for i, (n, dt) in enumerate(_shape_cases()):
        ins = []
        for r in range(world):
            g = torch.Generator().manual_seed(7000 + 100 * i + r)
            host = torch.randn(n + 1, generator=g).to(dt)
            ins.append((host[1:] if i % 2 else host[:n]).float())
        exp = sum(ins)
        tol = 1e-6 if dt == torch.float32 else 1e-2
        for r in range(world):
            got = torch.from_numpy(res[r][i])
            assert got.shape == exp.shape
            assert torch.allclose(got, exp, atol=tol * 4, rtol=tol), (i, n, dt, r)
    assert res[0]["over"] == res[1]["over"] == "refused"


# ----------------------------------------------------------------------------- DDP data plane
def _ddp_worker(rank, world, port, q, zero=False):
    """DDP with the automatic IPC route: the no-decay group (a 1-D weight, a few KiB) is
    all-reduced by the IPC kernels on a side stream, the 4 MiB decay group by the process group."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GRT_IPC_ALLOW_GLOO="1",
                      GRT_IPC_COLLECTIVES="auto", LOCAL_WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch.nn as nn
        from gke_ray_train_amd.parallel.ddp import DistributedDataParallel

        class Net(nn.Module):
            def __init__(self):
                super().__init__()
                self.fc1 = nn.Linear(1024, 1024, bias=False)
                self.norm = nn.Module()
                self.norm.weight = nn.Parameter(torch.ones(1024))

            def forward(self, x):
                return (self.fc1(x) * self.norm.weight).square().mean()

        torch.manual_seed(0)
        net = Net().cuda()
        ddp = DistributedDataParallel(net, broadcast_params=True, shard_optimizer=zero)
        g = torch.Generator().manual_seed(50 + rank)
        x = torch.randn(16, 1024, generator=g).cuda()
        ddp(x).backward()
        ddp.finish_gradient_sync()
        torch.cuda.synchronize()
        out = {"ipc": ddp.ipc_bucket_launches,
               "fc1": net.fc1.weight.grad.float().cpu().numpy(),
               "norm": net.norm.weight.grad.float().cpu().numpy()}
        if zero:  # this rank's reduced shard of every group (what the sharded AdamW consumes)
            out["shards"] = [sg.float().cpu().numpy() for sg in ddp.grad_buffers()]
            out["layout"] = [[(b.start, b.end, b.shard_off) for b in grp.buckets] for grp in ddp.groups]
        # the same gradients without DDP on this rank's data (summed over ranks by the parent)
        torch.manual_seed(0)
        ref = Net().cuda()
        ref(x).backward()
        out["ref_fc1"] = ref.fc1.weight.grad.float().cpu().numpy()
        out["ref_norm"] = ref.norm.weight.grad.float().cpu().numpy()
        q.put((rank, out))
    except Exception as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _ddp_zero_worker(rank, world, port, q):
    _ddp_worker(rank, world, port, q, zero=True)


@pytest.mark.parametrize("zero", [False, True])
def test_ddp_small_bucket_over_ipc(zero):
    """zero: the ZeRO engine's IPC bucket (all-reduce over IPC + this rank's chunk copied into the
    gradient shard on the side stream) gives the same shard as the reduce-scatter would."""
    world = 2
    res = _spawn(_ddp_zero_worker if zero else _ddp_worker, world)
    for k in ("fc1", "norm"):
        exp = sum(torch.from_numpy(res[r][f"ref_{k}"]) for r in range(world))
        for r in range(world):
            got = torch.from_numpy(res[r][k])
            assert torch.allclose(got, exp, atol=1e-5, rtol=1e-4), (k, r, (got - exp).abs().max())
    for r in range(world):
        assert res[r]["ipc"] >= 1, "the no-decay bucket did not take the IPC route"
    if zero:
        import numpy as np
        for r in range(world):
            full = {"fc1": sum(torch.from_numpy(res[k]["ref_fc1"]) for k in range(world)).reshape(-1),
                    "norm": sum(torch.from_numpy(res[k]["ref_norm"]) for k in range(world)).reshape(-1)}
            # one parameter per group: the shard is rank r's 1/world chunk of that parameter's summed
            # gradient (fc1: 1024 x 1024 over RCCL-path gloo, norm: 1024 over the IPC kernel)
            for shard, buckets in zip(res[r]["shards"], res[r]["layout"]):
                assert len(buckets) == 1 and np.isfinite(shard).all()
                c = (buckets[0][1] - buckets[0][0]) // world
                name = "fc1" if c * world >= 1024 * 1024 else "norm"
                exp = full[name][r * c:(r + 1) * c]
                got = torch.from_numpy(shard[:c])
                assert torch.allclose(got, exp, atol=1e-5, rtol=1e-4), (name, r, (got - exp).abs().max())


# ----------------------------------------------------------------------------- fail-stop
def _late_peer_worker(rank, world, port, q):
    """Rank 2 reaches the collective 6 s late against a 2 s IPC timeout. Every rank must end with a
    NaN (never a plausible) result and raise at its next check; later calls fail at once."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GRT_IPC_ALLOW_GLOO="1",
                      GRT_IPC_COLLECTIVES="auto", LOCAL_WORLD_SIZE=str(world), GRT_IPC_TIMEOUT_S="2")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        import torch.nn as nn
        from gke_ray_train_amd.parallel import ipc
        from gke_ray_train_amd.parallel.ddp import DistributedDataParallel

        class Net(nn.Module):
            def __init__(self):
                super().__init__()
                self.fc1 = nn.Linear(256, 256, bias=False)
                self.norm = nn.Module()
                self.norm.weight = nn.Parameter(torch.ones(256))

            def forward(self, x):
                return (self.fc1(x) * self.norm.weight).square().mean()

        torch.manual_seed(0)
        net = Net().cuda()
        ddp = DistributedDataParallel(net, broadcast_params=True)
        assert ddp._ipc is not None and ddp._ipc.timeout_s == 2.0
        # (1) a healthy step first: the IPC route works and check_all passes
        x = torch.randn(8, 256, device="cuda")
        with ddp.no_sync():  # library handles / first-call set-up outside the 2 s IPC window
            ddp(x).backward()
        torch.cuda.synchronize()
        ddp.zero_grad()
        dist.barrier()
        ddp(x).backward()
        ddp.finish_gradient_sync()
        torch.cuda.synchronize()
        ipc.check_all()
        out["healthy_finite"] = bool(torch.isfinite(net.norm.weight.grad).all())
        ddp.zero_grad()
        # (2) rank 2 is late: the IPC-routed bucket (norm weight) of every rank comes out NaN
        if rank == 2:
            time.sleep(6.0)
        ddp(x).backward()
        ddp.finish_gradient_sync()
        torch.cuda.synchronize()
        out["late_nan"] = bool(torch.isnan(net.norm.weight.grad).all())
        try:
            ipc.check_all()
            out["raised"] = None
        except RuntimeError as e:
            out["raised"] = str(e)
        # (3) the communicator stays failed: the next call returns NaN without waiting
        t0 = time.time()
        y = torch.ones(64, device="cuda")
        ddp._ipc.all_reduce(y)
        torch.cuda.synchronize()
        out["after_s"] = time.time() - t0
        out["after_nan"] = bool(torch.isnan(y).all())
        q.put((rank, out))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_late_peer_fails_every_rank_loudly():
    res = _spawn(_late_peer_worker, 3, timeout=240)
    for r in range(3):
        o = res[r]
        assert o["healthy_finite"], r
        assert o["late_nan"], f"rank {r} consumed a non-NaN result of a timed-out all-reduce"
        assert o["raised"] and "IPC collective failed" in o["raised"], (r, o["raised"])
        assert o["after_nan"] and o["after_s"] < 1.5, (r, o["after_s"])
    # the first rank to time out names the late rank and aborts the communicator for the others
    # (whose waits then end early); the late rank learns of the abort on arrival
    assert any("rank(s) [2]" in res[r]["raised"] for r in (0, 1)), [res[r]["raised"] for r in range(3)]
    assert "aborted" in res[2]["raised"]


def _self_test_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd.parallel.ipc import IpcCommunicator
        c = IpcCommunicator(max_bytes=8 << 20, timeout_s=20.0)
        ok = c.self_test()
        c.close()
        q.put((rank, {"ok": ok}))
    except Exception as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 8])
def test_self_test_against_process_group(world):
    """The set-up self-test (one- and two-shot, multi-block, 3 back-to-back calls per case, both
    dtypes, exact integer data against the process group's own all-reduce) passes on a healthy node."""
    res = _spawn(_self_test_worker, world)
    assert all(res[r]["ok"] for r in range(world))
