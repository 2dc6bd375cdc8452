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


@pytest.mark.parametrize("world", [2, 3])
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
