#!/usr/bin/env python3
"""Where a GEMM launch's time goes inside the graph-replayed B=256 round (diagnostics).

Needs a library built with -DCGL_GEMM_TRACE (bash tools/build_variant.sh trace -DCGL_GEMM_TRACE) selected by
CGL_LIB_PATH, and CGL_GEMM_TRACE=1: every GEMM workgroup stamps the 100 MHz wall clock at entry, k-loop start,
k-loop end and exit (cgl_gemm.hip).  After --rounds graph-replayed rounds the last round's stamps are read and
summarised per GEMM descriptor (plan order, CGL_PLAN_DEBUG=1 prints the descriptors):
  span        first kernel entry -> last exit of the problem's workgroups (us)
  ramp        first -> last workgroup entry (dispatch spread)
  entry_body  median kernel entry -> body start (descriptor search in the grouped launch)
  pro         median body start -> k-loop start (operand-transform prologue, epilogue-operand prefetch)
  first       median k-loop start -> chunk 0 consumed (the first operand round trip)
  kloop       median k-loop (incl. the in-workgroup split-K sum)
  epi         median k-loop end -> exit (split-K combine, epilogue, stores, BatchNorm partials)
  gap         this problem's first entry - the previous problem's last exit (launch boundary, us)

    CGL_LIB_PATH=cgl-gan_amd/lib_trace/libcglgan_hip.so CGL_GEMM_TRACE=1 python tools/gemm_trace.py
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cgl-gan_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--words", type=int, default=8, help="CGL_GEMM_TRACE_W of the build (72 with -DCGL_GEMM_TRACE_CHUNKS)")
    a = ap.parse_args()
    from cglgan import GanStep, specs
    from cglgan import _lib as C
    from cglgan.init import default_init
    os.environ["CGL_GEMM_TRACE"] = "1"
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.Generator(device="cuda").manual_seed(1000)
        real = torch.rand(60000, 784, device="cuda", generator=g) * 2 - 1
        gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
        st = GanStep(gm, dm, batch=a.batch, batch_real=a.batch, loss="ce", weighting="capgan", seed=20211212,
                     gen_z=True, real=real, sample_n=real.shape[0])
        torch.manual_seed(20211212)
        default_init(gm, st.g_views)
        torch.manual_seed(20211213)
        default_init(dm, st.d_views)
        st.reset()
        for r in range(a.rounds):
            st.run(graph=True)
        torch.cuda.synchronize()
        n = C.lib.cgl_gan_gemm_trace(st._h, None, 0)
        if n <= 0:
            raise SystemExit(f"no trace ({n}): build with -DCGL_GEMM_TRACE and set CGL_GEMM_TRACE=1")
        buf = (ctypes.c_ulonglong * n)()
        got = C.lib.cgl_gan_gemm_trace(st._h, buf, n)
        assert got == n, got
    W, NW = a.words, 4096    # CGL_GEMM_TRACE_W words per workgroup, CGL_GEMM_TRACE_WGS workgroups per problem
    rows, prev_end, t00 = [], None, None
    us = lambda x: x / 100.0      # 100 MHz ticks -> us
    med = lambda xs: round(us(statistics.median(xs)), 2) if xs else None
    for q in range(n // (W * NW)):
        ws = []
        for i in range(NW):
            t = list(buf[(q * NW + i) * W:(q * NW + i) * W + 6])
            if t[1] == 0:
                break
            ws.append(t)
        if not ws:
            continue
        t0 = min(w[0] for w in ws)
        t00 = t0 if t00 is None else t00
        ends = [w[5] for w in ws if w[5]]
        t_end = max(ends) if ends else max(w[4] for w in ws)
        first = [w for w in ws if w[3]]
        row = {"desc": q, "wgs": len(ws), "start": round(us(t0 - t00), 2), "span": round(us(t_end - t0), 2),
               "ramp": round(us(max(w[0] for w in ws) - t0), 2),
               "entry_body": med([w[1] - w[0] for w in ws]),       # descriptor search, wrapper
               "pro": med([w[2] - w[1] for w in ws]),              # operand-transform prologue, epilogue prefetch
               "first": med([w[3] - w[2] for w in first]),         # k-loop start -> chunk 0 consumed
               "kloop": med([w[4] - w[2] for w in ws]),
               "per_chunk_rest": None,
               "epi": med([w[5] - w[4] for w in ws if w[5]]),
               "gap": round(us(t0 - prev_end), 2) if prev_end is not None else None}
        if W > 8:     # per-chunk stamps of wave 0: median over workgroups of each chunk-to-chunk interval
            ch = []
            for i in range(len(ws)):
                base = (q * NW + i) * W
                ts = [buf[base + 8 + j] for j in range(W - 8)]
                ts = [t for t in ts if t]
                ch.append([ts[j + 1] - ts[j] for j in range(len(ts) - 1)])
            m = max(len(c) for c in ch) if ch else 0
            row["chunk_us"] = [round(us(statistics.median([c[j] for c in ch if len(c) > j])), 3) for j in range(m)]
        prev_end = t_end
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
