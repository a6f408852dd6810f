"""fp8 decode microbench (config #5): the gfx950 fp8 MFMA linear against the
bf16 hipBLASLt product (torch.matmul) on the Llama-3-8B decode shapes, then a
whole llama3-8b decode step (batch 8) on bf16 vs fp8 weights.

    python scripts/fp8_bench.py [--batch 8] [--iters 50] [--out gpurun_out/fp8_bench.jsonl]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pbs_amd.models.llama import PRESETS, LlamaDecoder  # noqa: E402
from pbs_amd.ops import llm  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--skip-model", action="store_true")
    ap.add_argument("--skip-linear", action="store_true")
    ap.add_argument("--variants", default="bf16,fp8,fp8+graph")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = open(a.out, "a") if a.out else None

    def emit(rec):
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
            out.flush()

    cfg = PRESETS["llama3-8b"]
    hd = cfg.head_dim
    shapes = {"qkv": ((cfg.n_heads + 2 * cfg.n_kv_heads) * hd, cfg.dim), "o": (cfg.dim, cfg.n_heads * hd),
              "w13": (2 * cfg.ffn_dim, cfg.dim), "w2": (cfg.dim, cfg.ffn_dim), "lm_head": (cfg.vocab, cfg.dim)}
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (N, K) in ({} if a.skip_linear else shapes).items():
        w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).bfloat16()
        x = torch.randn(a.batch, K, device="cuda", generator=g).bfloat16()
        W = llm.Fp8Weight(w)
        t16 = timeit(lambda: torch.matmul(x, w.t()), a.iters)
        t8 = timeit(lambda: llm.fp8_linear(x, W), a.iters)
        xq, sx = llm.quant_rows_fp8(x)
        y = torch.empty(a.batch, N, dtype=torch.bfloat16, device="cuda")
        L = llm.lib()
        tk = timeit(lambda: L.gpbs_hip_fp8_linear(llm._ptr(xq), llm._ptr(sx), llm._ptr(W.qs), llm._ptr(W.s),
                                                   llm._ptr(y), a.batch, N, K, llm._stream()), a.iters)
        var = {}
        for opt in range(4):  # kernel variants: bit0 non-temporal W loads, bit1 4 waves/WG
            L.gpbs_hip_fp8_set_opts(opt)
            var[f"opt{opt}"] = round(timeit(lambda: L.gpbs_hip_fp8_linear(
                llm._ptr(xq), llm._ptr(sx), llm._ptr(W.qs), llm._ptr(W.s), llm._ptr(y), a.batch, N, K,
                llm._stream()), a.iters), 2)
        L.gpbs_hip_fp8_set_opts(0)
        emit({"bench": "linear", "name": name, "variants_us": var, "M": a.batch, "N": N, "K": K, "bf16_us": round(t16, 2),
              "fp8_us": round(t8, 2), "fp8_kernel_us": round(tk, 2),
              "bf16_TBps": round(N * K * 2 / t16 / 1e6, 3), "fp8_kernel_TBps": round(N * K / tk / 1e6, 3),
              "speedup": round(t16 / t8, 3)})
        del w, W, x
    torch.cuda.empty_cache()
    if a.skip_model:
        return
    res = {}
    for fp8, graph in [(v.startswith("fp8"), v.endswith("+graph")) for v in a.variants.split(",")]:
        torch.manual_seed(0)
        t0 = time.perf_counter()
        dec = LlamaDecoder(cfg, batch=a.batch, context=1024, device="cuda", fp8=fp8, graph=graph)
        toks = torch.randint(0, cfg.vocab, (a.batch, 128), device="cuda")
        nxt = dec.prefill(toks)
        for _ in range(3):
            nxt = dec.decode_step(nxt)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(a.steps):
            nxt = dec.decode_step(nxt)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t1) / a.steps * 1e3
        key = ("fp8" if fp8 else "bf16") + ("+graph" if graph else "")
        res[key] = ms
        emit({"bench": "llama3-8b-decode", "weights": key, "batch": a.batch,
              "ms_per_token_step": round(ms, 3), "tok_per_s": round(a.batch * 1e3 / ms, 1),
              "setup_s": round(t1 - t0, 1)})
        del dec
        torch.cuda.empty_cache()
    if len(res) == 3:
        emit({"bench": "llama3-8b-decode", "speedup_fp8_vs_bf16": round(res["bf16"] / res["fp8"], 3),
              "speedup_fp8graph_vs_bf16": round(res["bf16"] / res["fp8+graph"], 3)})


if __name__ == "__main__":
    main()
