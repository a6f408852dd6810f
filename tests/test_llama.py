"""Llama-3 tenants (config #5): architecture, decode-with-cache consistency,
training progress (CPU, tiny preset), and the gfx950 fused decode kernels
against fp32 PyTorch references (GPU)."""
import pytest
import torch

from pbs_amd.models.llama import PRESETS, Llama, LlamaDecoder, LlamaTrainer, apply_rope_ref, rope_tables


def test_llama3_8b_parameter_count():
    n = PRESETS["llama3-8b"].n_params()
    assert 8.0e9 < n < 8.1e9, n


def test_decode_with_kv_cache_matches_full_forward():
    torch.manual_seed(0)
    cfg = PRESETS["tiny"]
    dec = LlamaDecoder(cfg, batch=2, context=64, device="cpu", dtype=torch.float32, fused=False)
    toks = torch.randint(0, cfg.vocab, (2, 12))
    nxt = dec.prefill(toks)
    seq = torch.cat([toks, nxt], dim=1)
    for _ in range(4):
        nxt = dec.decode_step(nxt)
        seq = torch.cat([seq, nxt], dim=1)
    # the cached greedy continuation equals an uncached forward of the same prefix
    full = dec.model(seq[:, :-1])
    assert torch.equal(full[:, -1].argmax(-1), seq[:, -1])


def test_training_step_reduces_loss():
    torch.manual_seed(0)
    tr = LlamaTrainer(PRESETS["tiny"], batch=4, seq=32, device="cpu", dtype=torch.float32, lr=3e-3)
    losses = [tr.step().item() for _ in range(8)]
    assert losses[-1] < losses[0] - 0.5, losses


@pytest.mark.gpu
def test_fused_llm_kernels_match_fp32_reference():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pbs_amd.ops import llm
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(37, 4096, device="cuda", generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(4096, device="cuda", generator=g)).bfloat16()
    xf = x.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    out = llm.rmsnorm(x, w, 1e-5)
    assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    a = torch.randn(8, 14336, device="cuda", generator=g).bfloat16()
    b = torch.randn(8, 14336, device="cuda", generator=g).bfloat16()
    ref = torch.nn.functional.silu(a.float()) * b.float()
    assert (llm.swiglu(a, b).float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    cfg = PRESETS["llama3-8b"]
    cos, sin = rope_tables(cfg, "cuda")
    q = torch.randn(2, 3, 32, 128, device="cuda", generator=g).bfloat16()
    ref = apply_rope_ref(q.float(), cos[100:103], sin[100:103])
    assert (llm.rope(q, cos, sin, 100).float() - ref).abs().max().item() < 3e-2


@pytest.mark.gpu
def test_fused_decoder_matches_eager_decoder():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)
    cfg = PRESETS["tiny"]
    d1 = LlamaDecoder(cfg, batch=2, context=64, device="cuda", fused=True)
    d2 = LlamaDecoder(cfg, batch=2, context=64, device="cuda", fused=False)
    d2.model.load_state_dict(d1.model.state_dict())
    toks = torch.randint(0, cfg.vocab, (2, 16), device="cuda")
    with torch.no_grad():
        l1 = d1.model(toks, fused=True)
        l2 = d2.model(toks, fused=False)
    assert (l1.float() - l2.float()).abs().max().item() < 5e-2 * l2.float().abs().max().item()
