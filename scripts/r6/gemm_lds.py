"""Do library GEMMs at the tiny-model shapes read stale LDS? Fill LDS with NaN / 0 before each."""
import sys, os, itertools
sys.path.insert(0, os.getcwd())
import torch
import torch.nn.functional as F
from gke_ray_train_amd import _native
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms
C = _native.kernels()
g = torch.Generator(device="cuda").manual_seed(0)
shapes = []
for (M, K, N) in [(256, 512, 1024), (256, 512, 512), (256, 512, 2752), (256, 1376, 512), (256, 512, 512 * 1),
                  (1280, 256, 512), (1280, 256, 256), (1280, 256, 1376), (1280, 688, 256), (256, 512, 64), (1280, 256, 512)]:
    shapes.append((M, K, N))
def run(pat, tuned):
    out = []
    for (M, K, N) in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
        for f in (lambda: F.linear(x, w), lambda: dy @ w, lambda: torch.mm(dy.t().contiguous(), x.t().contiguous().t()),
                  lambda: dy.t() @ x, lambda: F.linear(dy, w.t().contiguous())):
            C.lds_fill(pat, 0)
            out.append(f())
    torch.cuda.synchronize()
    return out
for tuned in (False, True):
    if tuned:
        print("tuned table:", enable_tuned_gemms())
    g.manual_seed(0); a = run(0x7FC00000, tuned)
    g.manual_seed(0); b = run(0, tuned)
    bad = [i for i, (x, y) in enumerate(zip(a, b)) if not (torch.isfinite(x).all() and torch.equal(x, y))]
    print("tuned" if tuned else "default", "GEMM results differing / non-finite under NaN LDS:", bad, flush=True)
