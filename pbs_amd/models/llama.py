"""Llama-3 family tenants (BASELINE config #5: "Llama-3-8B inference
co-located with a bf16 training tenant").

Random-initialised weights of the published architecture (no checkpoints
exist offline): GQA attention with RoPE (theta 500k), SwiGLU MLP, RMSNorm,
bf16 parameters and activations.  Two entry points:

* ``LlamaDecoder`` -- inference: prefill into a static KV cache sized for the
  full context, then one-token decode steps.  On a GPU the decode path runs
  the fused gfx950 kernels of ``pbs_amd.ops.llm`` (RMSNorm, SwiGLU, RoPE) and
  hipBLASLt for the projections; ``fused=False`` is the eager reference.
* ``LlamaTrainer`` -- training: causal-LM loss, backward, fused AdamW step
  (autograd through the PyTorch ops; bf16 weights, fp32 optimizer state).

Sizes are the real ones ("llama3-8b": 8.03 B parameters, 16 GB bf16); the
small presets exist for tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LlamaConfig:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    vocab: int = 128256
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq: int = 8192

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def n_params(self) -> int:
        hd = self.head_dim
        attn = self.dim * (self.n_heads * hd) * 2 + self.dim * (self.n_kv_heads * hd) * 2
        mlp = 3 * self.dim * self.ffn_dim
        return self.n_layers * (attn + mlp + 2 * self.dim) + 2 * self.vocab * self.dim + self.dim


PRESETS = {
    "llama3-8b": LlamaConfig(),
    "llama3-1b": LlamaConfig(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192),
    "tiny": LlamaConfig(dim=256, n_layers=2, n_heads=8, n_kv_heads=2, ffn_dim=512, vocab=1024, max_seq=256),
}


def rope_tables(cfg: LlamaConfig, device, dtype=torch.float32):
    hd = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, device=device, dtype=torch.float64) / hd))
    t = torch.arange(cfg.max_seq, device=device, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().to(dtype), f.sin().to(dtype)  # [max_seq, hd/2]


def apply_rope_ref(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, S, H, hd] (interleaved pairs), cos/sin [S, hd/2]."""
    xf = x.float().unflatten(-1, (-1, 2))
    a, b = xf[..., 0], xf[..., 1]
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    return torch.stack((a * c - b * s, a * s + b * c), dim=-1).flatten(-2).to(x.dtype)


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).to(x.dtype) * self.weight


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        hd = cfg.head_dim
        self.cfg = cfg
        self.attn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.wq = nn.Linear(cfg.dim, cfg.n_heads * hd, bias=False)
        self.wk = nn.Linear(cfg.dim, cfg.n_kv_heads * hd, bias=False)
        self.wv = nn.Linear(cfg.dim, cfg.n_kv_heads * hd, bias=False)
        self.wo = nn.Linear(cfg.n_heads * hd, cfg.dim, bias=False)
        self.mlp_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.w1 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)  # gate
        self.w3 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)  # up
        self.w2 = nn.Linear(cfg.ffn_dim, cfg.dim, bias=False)  # down

    def attention(self, h, cos, sin, cache=None, pos: int = 0, fused: bool = False):
        B, S, _ = h.shape
        cfg, hd = self.cfg, self.cfg.head_dim
        q = self.wq(h).view(B, S, cfg.n_heads, hd)
        k = self.wk(h).view(B, S, cfg.n_kv_heads, hd)
        v = self.wv(h).view(B, S, cfg.n_kv_heads, hd)
        if fused:
            from ..ops import llm
            q, k = llm.rope(q, cos, sin, pos), llm.rope(k, cos, sin, pos)
        else:
            q = apply_rope_ref(q, cos[pos:pos + S], sin[pos:pos + S])
            k = apply_rope_ref(k, cos[pos:pos + S], sin[pos:pos + S])
        if cache is not None:
            kc, vc = cache
            kc[:, :, pos:pos + S] = k.transpose(1, 2)
            vc[:, :, pos:pos + S] = v.transpose(1, 2)
            k_all, v_all = kc[:, :, :pos + S], vc[:, :, :pos + S]
        else:
            k_all, v_all = k.transpose(1, 2), v.transpose(1, 2)
        # GQA without materialising repeated K/V (at decode the cache read is
        # the attention cost; repeat_interleave would read+write it 4x more)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k_all, v_all, is_causal=(S > 1), enable_gqa=True)
        return self.wo(o.transpose(1, 2).reshape(B, S, cfg.n_heads * hd))

    def attach_fp8(self):
        """Quantise this block's linears to e4m3fn for the fp8 decode path:
        q/k/v packed into one [(H + 2 Hkv) hd, dim] weight, gate/up into one
        [2 ffn, dim] weight, so a decode step streams each layer in 4 launches."""
        from ..ops import llm
        self._fp8 = {
            "qkv": llm.Fp8Weight(torch.cat([self.wq.weight, self.wk.weight, self.wv.weight], 0)),
            "o": llm.Fp8Weight(self.wo.weight),
            "w13": llm.Fp8Weight(torch.cat([self.w1.weight, self.w3.weight], 0)),
            "w2": llm.Fp8Weight(self.w2.weight),
        }

    def forward_fp8(self, x, cos, sin, cache, pos: int):
        """Decode/prefill block on fp8 weights (fp8 MFMA linears + fused gfx950
        RMSNorm/RoPE/SwiGLU); inference only."""
        from ..ops import llm
        cfg, hd, f = self.cfg, self.cfg.head_dim, self._fp8
        B, S, _ = x.shape
        qkv = llm.fp8_linear_q(*llm.rmsnorm_quant_fp8(x, self.attn_norm.weight, self.attn_norm.eps), f["qkv"])
        nq, nkv = cfg.n_heads * hd, cfg.n_kv_heads * hd
        q = qkv[..., :nq].reshape(B, S, cfg.n_heads, hd)
        k = qkv[..., nq:nq + nkv].reshape(B, S, cfg.n_kv_heads, hd)
        v = qkv[..., nq + nkv:].reshape(B, S, cfg.n_kv_heads, hd)
        q, k = llm.rope(q, cos, sin, pos), llm.rope(k, cos, sin, pos)
        kc, vc = cache
        kc[:, :, pos:pos + S] = k.transpose(1, 2)
        vc[:, :, pos:pos + S] = v.transpose(1, 2)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), kc[:, :, :pos + S], vc[:, :, :pos + S],
                                           is_causal=(S > 1), enable_gqa=True)
        x = x + llm.fp8_linear(o.transpose(1, 2).reshape(B, S, nq), f["o"])
        gu = llm.fp8_linear_q(*llm.rmsnorm_quant_fp8(x, self.mlp_norm.weight, self.mlp_norm.eps), f["w13"])
        return x + llm.fp8_linear_q(*llm.swiglu_quant_fp8(gu), f["w2"])

    def decode_fp8_static(self, x, cos, sin, cache, pos_i32, pos_i64, mask):
        """One-token decode with every shape static and the position on device
        (capturable in a HIP graph): the KV row is written with index_copy_ at
        pos, and attention runs over the whole static cache with an additive
        mask, grouped per KV head (GQA without repeating K/V)."""
        from ..ops import llm
        cfg, hd, f = self.cfg, self.cfg.head_dim, self._fp8
        B = x.shape[0]
        G = cfg.n_heads // cfg.n_kv_heads
        qkv = llm.fp8_linear_q(*llm.rmsnorm_quant_fp8(x, self.attn_norm.weight, self.attn_norm.eps), f["qkv"])
        nq, nkv = cfg.n_heads * hd, cfg.n_kv_heads * hd
        kc, vc = cache
        if hd == 128 and G in (1, 2, 4, 8):  # fused gfx950 path: 2 launches between the qkv and o linears
            q = llm.qkv_rope_cache(qkv, cos, sin, pos_i32, kc, vc, cfg.n_heads)
            x = llm.fp8_linear_q(*llm.quant_rows_fp8(llm.decode_attn(q, kc, vc, pos_i32).view(B, 1, nq)), f["o"],
                                 resid=x)
            gu = llm.fp8_linear_q(*llm.rmsnorm_quant_fp8(x, self.mlp_norm.weight, self.mlp_norm.eps), f["w13"])
            return llm.fp8_linear_q(*llm.swiglu_quant_fp8(gu), f["w2"], resid=x)
        q = llm.rope_dpos(qkv[..., :nq].reshape(B, 1, cfg.n_heads, hd), cos, sin, pos_i32)
        k = llm.rope_dpos(qkv[..., nq:nq + nkv].reshape(B, 1, cfg.n_kv_heads, hd), cos, sin, pos_i32)
        v = qkv[..., nq + nkv:].reshape(B, 1, cfg.n_kv_heads, hd)
        kc.index_copy_(2, pos_i64, k.transpose(1, 2))
        vc.index_copy_(2, pos_i64, v.transpose(1, 2))
        qg = q.view(B, cfg.n_kv_heads, G, hd)
        sc = torch.matmul(qg, kc.transpose(-1, -2)).float() * (hd ** -0.5) + mask
        o = torch.matmul(torch.softmax(sc, -1).to(vc.dtype), vc)  # [B, Hkv, G, hd]
        x = x + llm.fp8_linear(o.reshape(B, 1, nq), f["o"])
        gu = llm.fp8_linear_q(*llm.rmsnorm_quant_fp8(x, self.mlp_norm.weight, self.mlp_norm.eps), f["w13"])
        return x + llm.fp8_linear_q(*llm.swiglu_quant_fp8(gu), f["w2"])

    def forward(self, x, cos, sin, cache=None, pos: int = 0, fused: bool = False):
        if fused:
            from ..ops import llm
            h = llm.rmsnorm(x, self.attn_norm.weight, self.attn_norm.eps)
            x = x + self.attention(h, cos, sin, cache, pos, fused=True)
            h = llm.rmsnorm(x, self.mlp_norm.weight, self.mlp_norm.eps)
            return x + self.w2(llm.swiglu(self.w1(h), self.w3(h)))
        x = x + self.attention(self.attn_norm(x), cos, sin, cache, pos)
        h = self.mlp_norm(x)
        return x + self.w2(F.silu(self.w1(h)) * self.w3(h))


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed = nn.Embedding(cfg.vocab, cfg.dim)
        self.layers = nn.ModuleList(Block(cfg) for _ in range(cfg.n_layers))
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.lm_head = nn.Linear(cfg.dim, cfg.vocab, bias=False)
        self._rope = None

    @torch.no_grad()
    def init_random(self, std: float = 0.02, seed: int = 0):
        g = torch.Generator(device=next(self.parameters()).device).manual_seed(seed)
        for n, p in self.named_parameters():
            if n.endswith("norm.weight"):
                p.fill_(1.0)
            else:
                p.normal_(0.0, std, generator=g)
        return self

    def rope(self, device):
        if self._rope is None or self._rope[0].device != device:
            self._rope = rope_tables(self.cfg, device)
        return self._rope

    def attach_fp8(self):
        """fp8 (e4m3fn) copies of every block linear and the LM head."""
        from ..ops import llm
        for layer in self.layers:
            layer.attach_fp8()
        self._fp8_head = llm.Fp8Weight(self.lm_head.weight)
        return self

    def forward_fp8(self, tokens, cache, pos: int = 0, last_only: bool = False):
        from ..ops import llm
        cos, sin = self.rope(tokens.device)
        x = self.embed(tokens)
        for i, layer in enumerate(self.layers):
            x = layer.forward_fp8(x, cos, sin, cache[i], pos)
        if last_only:
            x = x[:, -1:].contiguous()
        return llm.fp8_linear_q(*llm.rmsnorm_quant_fp8(x, self.norm.weight, self.norm.eps), self._fp8_head)

    def decode_fp8_static(self, tok, cache, pos_i32, pos_i64, mask):
        from ..ops import llm
        cos, sin = self.rope(tok.device)
        x = self.embed(tok)
        for i, layer in enumerate(self.layers):
            x = layer.decode_fp8_static(x, cos, sin, cache[i], pos_i32, pos_i64, mask)
        return llm.fp8_linear_q(*llm.rmsnorm_quant_fp8(x, self.norm.weight, self.norm.eps), self._fp8_head)

    def forward(self, tokens, cache=None, pos: int = 0, fused: bool = False, last_only: bool = False):
        cos, sin = self.rope(tokens.device)
        x = self.embed(tokens)
        for i, layer in enumerate(self.layers):
            x = layer(x, cos, sin, None if cache is None else cache[i], pos, fused)
        if last_only:
            x = x[:, -1:]
        x = self.norm(x) if not fused else __import__("pbs_amd.ops.llm", fromlist=["rmsnorm"]).rmsnorm(
            x, self.norm.weight, self.norm.eps)
        return self.lm_head(x)


def build(cfg: LlamaConfig, device, dtype) -> "Llama":
    """Construct directly in `dtype` on `device` (no fp32 transient: 8B
    parameters would otherwise pass through 32 GB of fp32)."""
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        with torch.device(device):
            m = Llama(cfg)
    finally:
        torch.set_default_dtype(prev)
    return m.init_random()


class LlamaDecoder:
    """Inference tenant: static KV cache, greedy decode."""

    def __init__(self, cfg: LlamaConfig, batch: int, context: int, device="cuda", dtype=torch.bfloat16,
                 fused: Optional[bool] = None, fp8: bool = False, graph: bool = False, static: bool = False):
        if not 0 < context <= cfg.max_seq:  # the RoPE tables cover max_seq positions
            raise ValueError(f"LlamaDecoder: context {context} must be in [1, max_seq={cfg.max_seq}]")
        self.cfg, self.batch, self.context = cfg, batch, context
        self.model = build(cfg, device, dtype)
        self.model.eval()
        self.fused = (torch.cuda.is_available() and str(device).startswith("cuda")) if fused is None else fused
        self.fp8 = fp8
        if fp8:  # weights streamed as e4m3fn through the fp8 MFMA linears (half the bytes of bf16)
            with torch.no_grad():
                self.model.attach_fp8()
        if (graph or static) and not fp8:
            raise ValueError("static-shape / graph decode is the fp8 path (needs fp8=True)")
        self.graph = graph
        self.static = static or graph  # static shapes + device position; graph=True also captures it
        self._g = self._step = None
        hd = cfg.head_dim
        self.cache = [(torch.zeros(batch, cfg.n_kv_heads, context, hd, device=device, dtype=dtype),
                       torch.zeros(batch, cfg.n_kv_heads, context, hd, device=device, dtype=dtype))
                      for _ in range(cfg.n_layers)]
        self.pos = 0

    @torch.no_grad()
    def prefill(self, tokens: torch.Tensor) -> torch.Tensor:
        self.pos = 0
        if self.fp8:
            logits = self.model.forward_fp8(tokens, self.cache, 0, last_only=True)
        else:
            logits = self.model(tokens, cache=self.cache, pos=0, fused=self.fused, last_only=True)
        self.pos = tokens.shape[1]
        return logits[:, -1].argmax(-1, keepdim=True)

    def _graph_setup(self, tok: torch.Tensor):
        """Build the static-shape step; with graph=True capture it (every launch
        of it) into a HIP graph, so later steps are one graph launch plus the
        position/token uploads."""
        dev = tok.device
        self._tok = tok.clone()
        self._pos_i32 = torch.zeros(1, dtype=torch.int32, device=dev)
        self._pos_i64 = torch.zeros(1, dtype=torch.int64, device=dev)
        self._ar = torch.arange(self.context, device=dev)

        def step():
            mask = torch.where(self._ar <= self._pos_i64, 0.0, float("-inf"))
            logits = self.model.decode_fp8_static(self._tok, self.cache, self._pos_i32, self._pos_i64, mask)
            return logits[:, -1].argmax(-1, keepdim=True)

        self._step = step
        if not self.graph:
            return
        self._set_pos()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):  # warm the allocator / library handles outside capture
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        self._g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g):
            self._out = step()

    def _set_pos(self):
        self._pos_i32.fill_(self.pos)
        self._pos_i64.fill_(self.pos)

    @torch.no_grad()
    def decode_step(self, tok: torch.Tensor) -> torch.Tensor:
        if self.pos >= self.context:
            self.pos = self.context // 2  # slide: keep the cache bounded for long runs
        if self.static:
            if self._step is None:
                self._graph_setup(tok)
            self._tok.copy_(tok)
            self._set_pos()
            if self.graph:
                self._g.replay()
                out = self._out.clone()
            else:
                out = self._step()
            self.pos += 1
            return out
        if self.fp8:
            logits = self.model.forward_fp8(tok, self.cache, self.pos)
        else:
            logits = self.model(tok, cache=self.cache, pos=self.pos, fused=self.fused)
        self.pos += 1
        return logits[:, -1].argmax(-1, keepdim=True)


class LlamaTrainer:
    """Training tenant: next-token loss, backward, fused AdamW (fp32 state)."""

    def __init__(self, cfg: LlamaConfig, batch: int, seq: int, device="cuda", dtype=torch.bfloat16, lr=1e-4):
        self.cfg, self.batch, self.seq = cfg, batch, seq
        self.model = build(cfg, device, dtype)
        self.model.train()
        kw = {"fused": True} if str(device).startswith("cuda") else {}
        self.opt = torch.optim.AdamW(self.model.parameters(), lr=lr, weight_decay=0.1, **kw)
        g = torch.Generator(device=device).manual_seed(1)
        self.tokens = torch.randint(0, cfg.vocab, (batch, seq + 1), device=device, generator=g)

    def step(self) -> torch.Tensor:
        x, y = self.tokens[:, :-1], self.tokens[:, 1:]
        logits = self.model(x)
        loss = F.cross_entropy(logits.float().reshape(-1, self.cfg.vocab), y.reshape(-1))
        loss.backward()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        return loss.detach()

    def tokens_per_step(self) -> int:
        return self.batch * self.seq

    def flops_per_step(self) -> float:
        return 6.0 * self.cfg.n_params() * self.tokens_per_step()
