"""KV-cache decode (models/generation.py) on the CPU: every greedy token equals the argmax of a full
no-cache forward over the prefix (cache writes, RoPE positions and the decode-step norm / projection
helpers agree with the training forward)."""
import torch

from gke_ray_train_amd.models import build_llama
from gke_ray_train_amd.models import generation as G


def test_greedy_decode_matches_full_forward():
    torch.manual_seed(0)
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32, seed=0).eval()
    ids = torch.randint(0, m.config.vocab_size, (2, 5))
    out = G.generate(m, ids, max_new_tokens=4)
    assert out.shape == (2, 9) and torch.equal(out[:, :5], ids)
    with torch.no_grad():
        for t in range(5, 9):
            logits = m(out[:, :t])["logits"][:, -1]
            assert torch.equal(logits.argmax(-1), out[:, t]), t


def test_cached_step_logits_match_full_forward():
    torch.manual_seed(1)
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32, seed=1).eval()
    ids = torch.randint(0, m.config.vocab_size, (1, 7))
    cache = G.KVCache(m.config, 1, 16, torch.device("cpu"), torch.float32)
    with torch.no_grad():
        G.forward_cached(m, ids[:, :6], cache)
        step = G.forward_cached(m, ids[:, 6:], cache)  # the one-token (S == 1) decode path
        full = m(ids)["logits"][:, -1].float()
    torch.testing.assert_close(step, full, rtol=1e-4, atol=1e-4)
