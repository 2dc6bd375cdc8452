# D = 128 RoPE kernel: bitwise tests against the generic kernel, isolated timing, interleaved headline A/B
O=gpurun_out/r6rope; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -k "rope" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 - > $O/time.log 2>&1 <<'PY' || { cat $O/time.log; exit 1; }
import torch, statistics
from gke_ray_train_amd import _native
from gke_ray_train_amd.ops import _ref
C = _native.kernels()
T, S, hq, hkv, D = 8192, 1024, 32, 32, 128
qkv = torch.randn(T, (hq + 2 * hkv) * D, device="cuda", dtype=torch.bfloat16)
cos, sin = _ref.rope_tables(S, D, 10000.0, device="cuda")
cos, sin = cos.float().contiguous(), sin.float().contiguous()
def t(fast, n=50):
    C.ew_set_fast(fast)
    for _ in range(5): C.rope_fwd(qkv, cos, sin, None, hq, hkv, D, S)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): C.rope_fwd(qkv, cos, sin, None, hq, hkv, D, S)
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3
r = {0: [], 1: []}
for _ in range(7):
    for f in (1, 0): r[f].append(t(f))
mb = 2 * 2 * T * (hq + hkv) * D / 1e6
for f in (1, 0):
    us = statistics.median(r[f]); print(f"rope_fwd fast={f}: {us:.1f} us  {mb / us:.2f} TB/s")
PY
cat $O/time.log
for i in 1 2 3; do
  for f in 1 0; do
    GRT_EW_FAST=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/b$f.$i.json 2> $O/b$f.$i.err || exit 1
    echo "ew_fast=$f round $i: $(python3 -c "import json;d=json.load(open('$O/b$f.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
