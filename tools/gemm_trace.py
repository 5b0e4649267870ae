"""Every GEMM of one training step (ops.GEMM_TRACE) with its operand strides, epilogue terms and the
kernel the library routes it to (alignn_gemm_path).  usage: python tools/gemm_trace.py [--batch B]
[--precision fp32|bf16] [--min-m M]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))
import alignn_mi355x as A  # noqa: E402
from alignn_mi355x import ops  # noqa: E402
from alignn_mi355x.synthetic import mp_like_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--precision", default="fp32")
ap.add_argument("--min-m", type=int, default=0)
ap.add_argument("--time", action="store_true", help="also time each call alone (HIP events, median of 7) and sort by time")
a = ap.parse_args()
torch.manual_seed(0)
model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to("cuda")
tr = A.FusedTrainer(model, precision=a.precision)
b = mp_like_batch(a.batch).to("cuda")
tr.forward_backward(b, 1)
torch.cuda.synchronize()
ops.GEMM_TRACE = []
tr.forward_backward(b, 2)
torch.cuda.synchronize()
calls, ops.GEMM_TRACE = ops.GEMM_TRACE, None
bf = ops.GEMM_BF16 if a.precision == "bf16" else 0
rows = []
for i, c in enumerate(calls):
    if c["A"].size(-2) < a.min_m:
        continue
    kw = {k: c[k] for k in ("alpha", "beta", "bias", "rowscale", "bias2", "relu", "mask", "reduce_batch", "c_rows",
                            "rowsum")}
    path = ops.gemm(c["A"], c["B"], c["C"], tile=bf, path_only=True, **kw)
    us = 0.0
    if a.time:
        C = c["C"].clone() if c["beta"] == 0 else c["C"]
        rs = kw.pop("rowsum")
        rs = rs.clone() if rs is not None else None
        ts = []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.gemm(c["A"], c["B"], C, tile=bf, rowsum=rs, **kw)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        us = sorted(ts[1:])[3]
        kw["rowsum"] = rs
    dt = "".join(n for t, n in ((c["A"], "A"), (c["B"], "B"), (c["C"], "C")) if t.dtype == torch.bfloat16)
    rows.append((us, f"{i:3d} {us:8.1f}us path={path} A{tuple(c['A'].shape)}{tuple(c['A'].stride())} "
                     f"B{tuple(c['B'].shape)}{tuple(c['B'].stride())} C{tuple(c['C'].shape)}{tuple(c['C'].stride())} "
                     f"bf16[{dt}] beta={c['beta']} bias={c['bias'] is not None} relu={c['relu']} "
                     f"mask={None if c['mask'] is None else tuple(c['mask'].stride())} rows={c['c_rows'] is not None} "
                     f"rowscale={c['rowscale'] is not None} rowsum={c['rowsum'] is not None} rb={c['reduce_batch']}"))
if a.time:
    rows.sort(key=lambda r: -r[0])
    print(f"total {sum(r[0] for r in rows):.1f} us over {len(rows)} calls")
for _, line in rows:
    print(line)
