"""SFT checkpoint robustness (CPU): a checkpoint failure on one rank raises on EVERY rank instead
of leaving the others blocked in a collective (gloo, world 2), and the RNG snapshot written to
``rng_state_<rank>.pth`` round-trips through ``torch.load(weights_only=True)`` and resumes the
streams — including the CPU generator the dropout kernels draw their seeds from."""
import os
import random
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd.trainer.sft import _rank_uniform_error
        out = []
        # 1) nobody failed: no raise, and the exchange leaves the group usable
        _rank_uniform_error(None, world, "ckpt")
        out.append("ok")
        # 2) only rank 0 failed: both ranks raise (rank 1 names "another rank")
        try:
            _rank_uniform_error(OSError("disk full") if rank == 0 else None, world, "ckpt")
            out.append("no-raise")
        except RuntimeError as e:
            out.append(str(e))
        dist.barrier()  # still reachable: nobody is stuck
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_checkpoint_failure_raises_on_every_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == ["ok", "ckpt failed"]
    assert res[1] == ["ok", "ckpt failed on another rank"]


def test_rng_snapshot_roundtrip_weights_only(tmp_path):
    from gke_ray_train_amd.ops.fused import dropout_seed_offset
    from gke_ray_train_amd.trainer.sft import _rng_restore, _rng_snapshot
    torch.manual_seed(5)
    random.seed(5)
    np.random.seed(5)
    torch.rand(3)
    path = tmp_path / "rng_state_0.pth"
    torch.save(_rng_snapshot(), path)
    expect = (random.random(), float(np.random.rand()), torch.rand(2), dropout_seed_offset(torch.empty(4)))
    torch.manual_seed(99)
    random.seed(99)
    np.random.seed(99)
    _rng_restore(torch.load(path, weights_only=True))
    got = (random.random(), float(np.random.rand()), torch.rand(2), dropout_seed_offset(torch.empty(4)))
    assert got[0] == expect[0] and got[1] == expect[1]
    assert torch.equal(got[2], expect[2])
    assert got[3] == expect[3]  # the resumed run draws the same dropout seed, not step 0's


def test_dropout_seed_offset_follows_cpu_rng():
    from gke_ray_train_amd.ops.fused import dropout_seed_offset
    torch.manual_seed(1)
    a = dropout_seed_offset(torch.empty(8))
    b = dropout_seed_offset(torch.empty(8))
    torch.manual_seed(1)
    assert dropout_seed_offset(torch.empty(8)) == a
    assert a != b and a[1] == 0 and 0 <= a[0] < 2 ** 62


def test_rng_state_legacy_and_hf_layouts_resume(tmp_path):
    """rng_state_<rank>.pth holding np.random.get_state() as a tuple with an ndarray (HF layout and
    this repo's pre-round-3 files) resumes through the weights-only loader with numpy's array
    globals allow-listed; an unreadable file is skipped with a warning."""
    import random
    import warnings

    import numpy as np
    import torch

    from gke_ray_train_amd.trainer.sft import _rng_load, _rng_restore
    st = np.random.get_state()
    p = tmp_path / "rng_state_0.pth"
    torch.save({"python": random.getstate(), "numpy": st, "cpu": torch.get_rng_state()}, str(p))
    rng = _rng_load(str(p))
    assert rng is not None
    np.random.rand(7)
    _rng_restore(rng)
    a = np.random.rand(4)
    np.random.set_state(st)
    assert (a == np.random.rand(4)).all()
    p.write_bytes(b"not a checkpoint")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert _rng_load(str(p)) is None
    assert any("cannot restore RNG state" in str(x.message) for x in w)
