"""fp8 (OCP e4m3fn) linears for the Llama inference tenant (config #5, CDNA4
fp8 MFMA; csrc/hip/fp8_kernels.hip).  CPU: the fp32 reference semantics.
GPU: the quantiser is checked bit-for-bit against PyTorch's e4m3fn cast and the
MFMA linear against the fp32 product of the same quantised operands."""
import pytest
import torch

from pbs_amd.models.llama import PRESETS, LlamaDecoder
from pbs_amd.ops import llm


def test_fp8_reference_semantics_cpu():
    torch.manual_seed(0)
    w = torch.randn(64, 512).bfloat16()
    W = llm.Fp8Weight(w)
    assert W.q.dtype == torch.float8_e4m3fn and W.s.shape == (64,)
    # every row uses the full e4m3 range: max |q| == 448
    assert torch.all(W.q.float().abs().amax(1) == llm.FP8_MAX)
    x = torch.randn(5, 512).bfloat16()
    ref = x.float() @ w.float().t()
    y = llm.fp8_linear_ref(x, W)
    rel = (y - ref).norm() / ref.norm()
    assert rel < 0.06, rel
    # a zero row gets scale 1 and zero output (no division by zero)
    y0 = llm.fp8_linear_ref(torch.zeros(1, 512).bfloat16(), W)
    assert torch.all(y0 == 0)
    with pytest.raises(ValueError):
        llm.Fp8Weight(torch.randn(10, 512))


@pytest.mark.gpu
def test_quant_rows_fp8_bit_exact():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.randn(67, 4096, device="cuda", generator=g) * 3).bfloat16()
    x[3] = 0
    q, s = llm.quant_rows_fp8(x)
    qr, sr = llm.quant_rows_fp8_ref(x)
    torch.testing.assert_close(s, sr, rtol=1e-6, atol=0)
    bad = q.view(torch.uint8) != qr.view(torch.uint8)
    mism = bad.float().mean().item()
    ex = [(x[i, j].item() / sr[i].item(), q[i, j].item(), qr[i, j].item()) for i, j in bad.nonzero()[:6].tolist()]
    # both round to nearest even; a disagreement is at most one e4m3 step (ties /
    # subnormal handling of the hardware convert)
    assert mism < 1e-2, (mism, ex)
    assert (q.float() - qr.float()).abs().max().item() <= 32  # at most one e4m3 step at the top binade


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (8, 6144, 4096), (17, 1024, 14336), (40, 256, 512),
                                   (64, 4096, 256), (100, 512, 1024)])
def test_fp8_linear_matches_fp32_reference(M, N, K):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = llm.Fp8Weight(w)
    y = llm.fp8_linear(x, W)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    xq, sx = llm.quant_rows_fp8(x)  # kernel operands -> fp32 product of exactly those
    ref = (xq.float() @ W.q.float().t()) * sx[:, None] * W.s[None, :]
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err  # fp32 accumulation order + bf16 output rounding
    # and close to the unquantised bf16 product
    full = x.float() @ w.float().t()
    assert ((y.float() - full).norm() / full.norm()).item() < 0.06


@pytest.mark.gpu
def test_fp8_decoder_tracks_bf16_decoder():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)
    cfg = PRESETS["tiny"]
    d16 = LlamaDecoder(cfg, batch=4, context=64, device="cuda", fused=True)
    d8 = LlamaDecoder(cfg, batch=4, context=64, device="cuda", fused=True, fp8=False)
    d8.model.load_state_dict(d16.model.state_dict())
    d8.model.attach_fp8()
    d8.fp8 = True
    toks = torch.randint(0, cfg.vocab, (4, 16), device="cuda")
    with torch.no_grad():
        l16 = d16.model(toks, cache=d16.cache, pos=0, fused=True)
        l8 = d8.model.forward_fp8(toks, d8.cache, 0)
        cos = torch.nn.functional.cosine_similarity(l8.float().flatten(1), l16.float().flatten(1)).min().item()
        assert cos > 0.98, cos
        # one cached decode step on each
        nxt = l16[:, -1].argmax(-1, keepdim=True)
        s16 = d16.model(nxt, cache=d16.cache, pos=16, fused=True)
        s8 = d8.model.forward_fp8(nxt, d8.cache, 16)
        cos = torch.nn.functional.cosine_similarity(s8.float().flatten(1), s16.float().flatten(1)).min().item()
        assert cos > 0.98, cos


@pytest.mark.gpu
def test_fused_norm_and_swiglu_quantisers_match_reference():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(9, 4096, device="cuda", generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(4096, device="cuda", generator=g)).bfloat16()
    q, s = llm.rmsnorm_quant_fp8(x, w, 1e-5)
    xf = x.float()
    h = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    qr, sr = llm.quant_rows_fp8_ref(h)
    torch.testing.assert_close(s, sr, rtol=1e-4, atol=0)
    deq, deqr = q.float() * s[:, None], qr.float() * sr[:, None]
    assert ((deq - deqr).norm() / deqr.norm()).item() < 0.01
    assert ((deq - h).norm() / h.norm()).item() < 0.05
    gu = torch.randn(5, 2 * 14336, device="cuda", generator=g).bfloat16()
    q, s = llm.swiglu_quant_fp8(gu)
    a, b = gu[:, :14336].float(), gu[:, 14336:].float()
    y = torch.nn.functional.silu(a) * b
    qr, sr = llm.quant_rows_fp8_ref(y)
    torch.testing.assert_close(s, sr, rtol=1e-3, atol=0)
    deq = q.float() * s[:, None]
    assert ((deq - y).norm() / y.norm()).item() < 0.05


@pytest.mark.gpu
def test_graph_captured_fp8_decode_matches_eager_fp8_decode():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)
    cfg = PRESETS["tiny"]
    de = LlamaDecoder(cfg, batch=4, context=64, device="cuda", fp8=True)
    toks = torch.randint(0, cfg.vocab, (4, 12), device="cuda")
    ne = de.prefill(toks)
    # the static-shape step (index_copy_ KV write, masked whole-cache GQA attention,
    # device-position RoPE) against the sliced eager fp8 step, on logits
    with torch.no_grad():
        pos_i32 = torch.full((1,), 12, dtype=torch.int32, device="cuda")
        pos_i64 = pos_i32.long()
        mask = torch.where(torch.arange(64, device="cuda") <= pos_i64, 0.0, float("-inf"))
        cache_s = [(k.clone(), v.clone()) for k, v in de.cache]
        ls = de.model.decode_fp8_static(ne, cache_s, pos_i32, pos_i64, mask)
        le = de.model.forward_fp8(ne, de.cache, 12)
    cos = torch.nn.functional.cosine_similarity(ls.float().flatten(1), le.float().flatten(1)).min().item()
    assert cos > 0.995, cos
    # layer 0's new KV row depends only on the embedding: same kernels, same values
    # (deeper layers inherit the attention-path rounding difference)
    (k1, v1), (k2, v2) = cache_s[0], de.cache[0]
    assert (k1.float() - k2.float()).abs().max().item() < 1e-2
    assert (v1.float() - v2.float()).abs().max().item() < 1e-2
    # graph replay == the same static step run eagerly (identical kernels); head_dim
    # 128 so the fused RoPE/cache + decode-attention kernels are the ones captured
    from pbs_amd.models.llama import LlamaConfig
    cfg = LlamaConfig(dim=512, n_layers=2, n_heads=4, n_kv_heads=1, ffn_dim=1024, vocab=1024, max_seq=256)
    de = LlamaDecoder(cfg, batch=4, context=64, device="cuda", fp8=True)
    ds = LlamaDecoder(cfg, batch=4, context=64, device="cuda", fp8=True, static=True)
    dg = LlamaDecoder(cfg, batch=4, context=64, device="cuda", fp8=True, graph=True)
    ds.model.load_state_dict(de.model.state_dict())
    dg.model.load_state_dict(de.model.state_dict())
    ds.model.attach_fp8()
    dg.model.attach_fp8()
    a, b = ds.prefill(toks), dg.prefill(toks)
    for _ in range(8):
        a, b = ds.decode_step(a), dg.decode_step(a)
        assert torch.equal(a, b)
    assert dg._g is not None and dg.pos == ds.pos == 20


@pytest.mark.gpu
def test_fused_decode_rope_cache_and_attention_match_reference():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pbs_amd.models.llama import LlamaConfig, apply_rope_ref, rope_tables
    cfg = LlamaConfig(dim=1024, n_layers=2, n_heads=8, n_kv_heads=2, ffn_dim=2048, vocab=1024, max_seq=256)
    g = torch.Generator(device="cuda").manual_seed(2)
    B, H, Hkv, hd, Cn, pos = 3, 8, 2, 128, 200, 137
    cos, sin = rope_tables(cfg, "cuda")
    kc = torch.randn(B, Hkv, Cn, hd, device="cuda", generator=g).bfloat16()
    vc = torch.randn(B, Hkv, Cn, hd, device="cuda", generator=g).bfloat16()
    k0, v0 = kc.clone(), vc.clone()
    qkv = torch.randn(B, 1, (H + 2 * Hkv) * hd, device="cuda", generator=g).bfloat16()
    pos_t = torch.full((1,), pos, dtype=torch.int32, device="cuda")
    q = llm.qkv_rope_cache(qkv, cos, sin, pos_t, kc, vc, H)
    qr = apply_rope_ref(qkv[..., :H * hd].float().view(B, 1, H, hd), cos[pos:pos + 1], sin[pos:pos + 1])
    kr = apply_rope_ref(qkv[..., H * hd:(H + Hkv) * hd].float().view(B, 1, Hkv, hd), cos[pos:pos + 1],
                        sin[pos:pos + 1])
    assert (q.float() - qr[:, 0]).abs().max().item() < 3e-2
    assert (kc[:, :, pos].float() - kr[:, 0]).abs().max().item() < 3e-2
    assert torch.equal(vc[:, :, pos], qkv[..., (H + Hkv) * hd:].view(B, Hkv, hd))
    others = torch.ones(Cn, dtype=torch.bool, device="cuda")
    others[pos] = False
    assert torch.equal(kc[:, :, others], k0[:, :, others]) and torch.equal(vc[:, :, others], v0[:, :, others])
    out = llm.decode_attn(q, kc, vc, pos_t)
    G = H // Hkv
    qf = q.float().view(B, Hkv, G, hd)
    sc = qf @ kc[:, :, :pos + 1].float().transpose(-1, -2) * hd ** -0.5
    ref = (torch.softmax(sc, -1) @ vc[:, :, :pos + 1].float()).reshape(B, H * hd)
    assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    # short prefix (fewer keys than one wave) and pos 0
    for p, ns in ((0, None), (5, None), (63, 4), (64, 3), (199, 1), (199, 8), (130, 2)):
        pos_t.fill_(p)
        out = llm.decode_attn(q, kc, vc, pos_t, nsplit=ns)
        sc = qf @ kc[:, :, :p + 1].float().transpose(-1, -2) * hd ** -0.5
        ref = (torch.softmax(sc, -1) @ vc[:, :, :p + 1].float()).reshape(B, H * hd)
        assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item(), (p, ns)


@pytest.mark.gpu
def test_fp8_linear_fused_residual():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator(device="cuda").manual_seed(9)
    W = llm.Fp8Weight((torch.randn(4096, 4096, device="cuda", generator=g) * 0.02).bfloat16())
    x = torch.randn(8, 1, 4096, device="cuda", generator=g).bfloat16()
    r = torch.randn(8, 1, 4096, device="cuda", generator=g).bfloat16()
    xq, sx = llm.quant_rows_fp8(x)
    y = llm.fp8_linear_q(xq, sx, W, resid=r)
    ref = llm.fp8_linear_q(xq, sx, W).float() + r.float()
    assert (y.float() - ref).abs().max().item() < 3e-2


def test_fp8_weight_lane_order_layout_cpu():
    """The pre-shuffled layout the MFMA kernel streams: lane l = 16 g + r of the
    wave owning (strip, block) reads W[16 strip + r][256 block + 64 u + 16 g : +16]
    at step u from one contiguous 1 KiB run."""
    torch.manual_seed(1)
    w = torch.randn(48, 768).bfloat16()
    W = llm.Fp8Weight(w)
    q, _ = llm.quant_rows_fp8_ref(w)
    assert torch.equal(W.q.view(torch.uint8), q.view(torch.uint8))  # unshuffle round-trips
    flat, rm = W.qs.view(torch.uint8).reshape(-1), q.view(torch.uint8)
    nkb = 768 // 256
    for strip, kb, u, lane in ((0, 0, 0, 0), (1, 2, 3, 63), (2, 1, 2, 17), (2, 2, 1, 40)):
        g, r = lane // 16, lane % 16
        off = ((strip * nkb + kb) * 4 + u) * 1024 + lane * 16
        k0 = 256 * kb + 64 * u + 16 * g
        assert torch.equal(flat[off:off + 16], rm[16 * strip + r, k0:k0 + 16])
