"""IPC data-plane routing and the IPC all-reduce protocol, on the CPU.

* routing: which messages go over the xGMI IPC kernels (parallel/ipc.py) is a pure function of
  (bytes, dtype, mode) -- identical on every rank, so no rank can take RCCL while a peer waits in
  the IPC kernel;
* set-up agreement: a rank that cannot export / open IPC handles, or a group whose ranks asked for
  different buffer sizes, makes EVERY rank raise (gloo, world 2, fake native layer) instead of
  leaving the healthy ranks blocked in a collective;
* protocol: a step-by-step model of the kernel's epoch / parity protocol
  (csrc/kernels/ipc_comm.hip header) under random interleavings of the ranks, including epoch
  wrap-around at 2^32: every staging / result read sees the data of its own call, and a
  single-buffered variant of the same protocol is caught by the same checker.
"""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gke_ray_train_amd.parallel import ipc


def test_routing_is_pure_and_mode_driven(monkeypatch):
    monkeypatch.delenv("GRT_IPC_COLLECTIVES", raising=False)
    assert ipc.ipc_mode() == "auto"
    cap = 8 << 20
    lim = ipc.route_limit("auto", cap)
    assert lim == ipc.IPC_AUTO_BYTES
    assert ipc.routes(4, torch.float32, lim)
    assert ipc.routes(lim, torch.bfloat16, lim)
    assert not ipc.routes(lim + 2, torch.bfloat16, lim)
    assert not ipc.routes(64, torch.float64, lim)
    assert not ipc.routes(0, torch.float32, lim)
    assert ipc.route_limit("1", cap) == cap and ipc.route_limit("0", cap) == 0
    assert not ipc.routes(4, torch.float32, ipc.route_limit("0", cap))
    for v, m in (("0", "0"), ("off", "0"), ("1", "1"), ("on", "1"), ("auto", "auto"), ("bogus", "auto")):
        monkeypatch.setenv("GRT_IPC_COLLECTIVES", v)
        assert ipc.ipc_mode() == m


def test_no_group_no_communicator():
    assert not (dist.is_available() and dist.is_initialized())
    assert ipc.communicator(None, "t") is None
    assert not ipc.ipc_available()


# ----------------------------------------------------------------------------- set-up agreement
class _FakeKernels:
    IPC_MAX_RANKS = 8
    IPC_SIGNAL_BYTES = 4096

    def __init__(self, rank, fail):
        self.rank, self.fail, self.n = rank, fail, 0

    def ipc_alloc(self, nbytes, fine, dev):
        self.n += 1
        return 0x1000 * self.n

    def ipc_handle(self, p, dev):
        if self.fail == ("export", self.rank):
            raise RuntimeError("hipIpcGetMemHandle: invalid argument")
        return bytes([self.rank]) * 64

    def ipc_open(self, h, dev):
        if self.fail == ("open", self.rank):
            raise RuntimeError("hipIpcOpenMemHandle failed")
        return 0x9000

    def ipc_close(self, p, dev):
        pass

    def ipc_free(self, p, dev):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup_worker(rank, world, port, fail, caps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd import _native
        _native.kernels = lambda: _FakeKernels(rank, fail)
        try:
            c = ipc.IpcCommunicator(max_bytes=caps[rank], device=torch.device("cpu"))
            q.put((rank, "ok", c.cap))
        except Exception as e:  # noqa: BLE001
            q.put((rank, "raised", str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail,caps", [(None, (4096, 4096)), (("export", 1), (4096, 4096)),
                                       (("open", 0), (4096, 4096)), (None, (4096, 8192))])
def test_setup_failure_is_agreed_by_every_rank(fail, caps):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_setup_worker, args=(r, 2, port, fail, caps, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, st, info = q.get(timeout=60)  # a split decision would hang here, not fail
            res[r] = (st, info)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    want = "ok" if fail is None and caps[0] == caps[1] else "raised"
    assert {r: st for r, (st, _) in res.items()} == {0: want, 1: want}, res
    if caps[0] != caps[1]:
        assert "sizes differ" in res[0][1] and "sizes differ" in res[1][1]


# ----------------------------------------------------------------------------- protocol model
class _Violation(AssertionError):
    pass


def _run_protocol(world, calls, seed, parities=2, two_shot=False, epoch0=0):
    """Ranks run as generators over shared state; the scheduler picks a random runnable rank at
    every step. A read checks the version (epoch) stamped on the data it reads."""
    rng = random.Random(seed)
    M32 = 0xFFFFFFFF
    staging = [[None] * parities for _ in range(world)]   # (epoch, values)
    result = [[None] * parities for _ in range(world)]    # per parity: {sub: (epoch, values)}
    signal = [[[0] * world for _ in range(2)] for _ in range(world)]  # [rank][phase][src]
    for r in range(world):
        for ph in range(2):
            for s in range(world):
                signal[r][ph][s] = epoch0 & M32
    outs = [[None] * len(calls) for _ in range(world)]

    def arrived(r, ph, e):
        return all(((signal[r][ph][p] - e) & M32) < 0x80000000 for p in range(world))

    def rank_prog(r):
        e = epoch0
        for ci, inputs in enumerate(calls):
            e = (e + 1) & M32
            par = e % parities
            x = inputs[r]
            staging[r][par] = (e, list(x))
            yield
            for p in range(world):  # start flag on every rank
                signal[p][0][r] = e
                yield
            while not arrived(r, 0, e):
                yield "blocked"
            n = len(x)
            if not two_shot:
                acc = [0.0] * n
                for p in range(world):
                    ver, vals = staging[p][par]
                    if ver != e:
                        raise _Violation(f"rank {r} call {ci} read rank {p}'s staging of epoch {ver}")
                    acc = [a + v for a, v in zip(acc, vals)]
                    yield
                outs[r][ci] = acc
                continue
            lo, hi = n * r // world, n * (r + 1) // world
            part = [0.0] * (hi - lo)
            for p in range(world):
                ver, vals = staging[p][par]
                if ver != e:
                    raise _Violation(f"rank {r} call {ci} read rank {p}'s staging of epoch {ver}")
                part = [a + v for a, v in zip(part, vals[lo:hi])]
                yield
            result[r][par] = {"epoch": e, "vals": part}
            yield
            for p in range(world):  # mid flag
                signal[p][1][r] = e
                yield
            while not arrived(r, 1, e):
                yield "blocked"
            acc = []
            for p in range(world):
                rp = result[p][par]
                if rp["epoch"] != e:
                    raise _Violation(f"rank {r} call {ci} read rank {p}'s result of epoch {rp['epoch']}")
                acc += rp["vals"]
                yield
            outs[r][ci] = acc

    progs = {r: rank_prog(r) for r in range(world)}
    steps = 0
    while progs:
        r = rng.choice(list(progs))
        try:
            next(progs[r])
        except StopIteration:
            del progs[r]
        steps += 1
        if steps > 10_000_000:
            raise AssertionError("protocol did not terminate")
    return outs


def _calls(world, n_calls, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n_calls):
        n = rng.choice([1, 3, 8, 13])
        out.append([[float(rng.randint(-9, 9)) for _ in range(n)] for _ in range(world)])
    return out


@pytest.mark.parametrize("two_shot", [False, True])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_epoch_parity_protocol_model(world, two_shot):
    calls = _calls(world, 12, world)
    for seed in range(30 if world < 8 else 8):
        for epoch0 in (0, 0xFFFFFFFF - 5):  # wrap-around of the 32-bit epoch inside the run
            outs = _run_protocol(world, calls, seed, two_shot=two_shot, epoch0=epoch0)
            for ci, inputs in enumerate(calls):
                exp = [sum(v) for v in zip(*inputs)]
                for r in range(world):
                    assert outs[r][ci] == exp, (seed, ci, r)


def test_single_buffer_variant_is_caught():
    """Without the parity double-buffer a fast rank overwrites its staging while a slow peer still
    reads the previous call: the checker must see it for some interleaving."""
    world = 3
    calls = _calls(world, 12, 7)
    caught = 0
    for seed in range(200):
        try:
            _run_protocol(world, calls, seed, parities=1)
        except _Violation:
            caught += 1
    assert caught > 0
