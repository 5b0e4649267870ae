"""GEMM plan tuning: records every ops.gemm call of one training step (bench workload), then replays
each distinct call under forced plans (tile shape x split-K) and the automatic plan, timing each with
HIP events (median of R reps).  Prints per-shape times and the best plan, plus the step totals.

usage: python tools/gemm_bench.py [--reps 15] [--json out.json]
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))
import alignn_mi355x as A  # noqa: E402
from alignn_mi355x import ops  # noqa: E402
from alignn_mi355x.synthetic import mp_like_batch  # noqa: E402

AUTO = -1
TILES = {AUTO: "auto"}
TILES.update({b + k: f"{s}/bk{bk}" for k, s in ((1, "128x128"), (2, "128x64"), (3, "64x128"), (4, "64x64"))
         for b, bk in ((0, "auto"), (16, 32), (32, 16), (128, 64))})


def timeit(fn, reps):
    """Device time per call: ``reps`` calls captured in one HIP graph (no host launch cost in the
    measurement), replayed 3 times between two events; median replay / reps."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return sorted(ts)[1]


def sig(c):
    A, B, C = c["A"], c["B"], c["C"]
    return (tuple(A.shape), tuple(A.stride()), tuple(B.shape), tuple(B.stride()), tuple(C.shape), tuple(C.stride()),
            c["beta"] != 0, c["reduce_batch"], c["c_rows"] is not None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--json")
    ap.add_argument("--quick", action="store_true", help="auto plan + torch.matmul (hipBLASLt/rocBLAS) only")
    ap.add_argument("--flag", type=int, default=0,
                    help="also time the auto plan with these tile flag bits ORed in (e.g. 1024: ALIGNN_GEMM_KW2) "
                         "and report its result's max difference from the auto plan's")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: the step's products with bf16 matrix-core inputs (config C3); the library "
                         "reference is then torch.matmul on bf16 copies of the operands")
    ap.add_argument("--min-m", type=int, default=0, help="only products with at least this many rows")
    ap.add_argument("--splits", default="1,2,4,8,16,32,64", help="split-K counts the forced plans try")
    a = ap.parse_args()
    splits = [int(x) for x in a.splits.split(",")]
    dev = "cuda"
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(dev)
    tr = A.FusedTrainer(model, precision=a.precision)
    bf = ops.GEMM_BF16 if a.precision == "bf16" else 0
    b = mp_like_batch(a.batch).to(dev)
    tr.forward_backward(b, 1)
    torch.cuda.synchronize()
    ops.GEMM_TRACE = []
    tr.forward_backward(b, 2)
    torch.cuda.synchronize()
    calls = ops.GEMM_TRACE
    ops.GEMM_TRACE = None
    groups = collections.OrderedDict()
    for c in calls:
        groups.setdefault(sig(c), []).append(c)
    print(f"{len(calls)} gemm calls, {len(groups)} distinct", flush=True)
    res = []
    tot_auto = tot_best = tot_lib = 0.0
    for key, cs in groups.items():
        c = cs[0]
        if c["A"].shape[-2] < a.min_m:
            continue
        C_save = c["C"].clone()

        def run(tile=0, split=None, c=c):
            ops.gemm(c["A"], c["B"], c["C"], alpha=c["alpha"], beta=c["beta"], bias=c["bias"], rowscale=c["rowscale"],
                     bias2=c["bias2"], relu=c["relu"], mask=c["mask"], reduce_batch=c["reduce_batch"],
                     c_rows=c["c_rows"], split_k=split, tile=tile | bf)

        t_auto = timeit(lambda: run(), a.reps)
        # library reference: the same plain product through torch.matmul (no epilogue)
        Am, Bm = c["A"], c["B"]
        if c["reduce_batch"]:
            Am = Am.transpose(0, 1).reshape(Am.shape[1], -1) if Am.dim() == 3 else Am
            Bm = Bm.reshape(-1, Bm.shape[-1]) if Bm.dim() == 3 else Bm
        if bf:
            Am, Bm = Am.bfloat16(), Bm.bfloat16()
        try:
            t_lib = timeit(lambda: torch.matmul(Am, Bm), a.reps)
        except Exception:  # noqa: BLE001
            t_lib = float("nan")
        extra = ""
        if a.flag:
            c["C"].copy_(C_save)
            run()
            ref = c["C"].clone()
            c["C"].copy_(C_save)
            run(a.flag)
            diff = float((c["C"] - ref).abs().max() / ref.abs().max().clamp(min=1e-30))
            t_flag = timeit(lambda: run(a.flag), a.reps)
            extra = f"  flag{a.flag} {t_flag:7.1f}us (diff {diff:.1e})"
            tot_flag = globals().setdefault("_tot_flag", [0.0])
            tot_flag[0] += t_flag * len(cs)
        trials = {}
        for tile in ([] if a.quick else sorted(TILES)):
            if tile < 16:
                continue
            for split in splits:
                try:
                    trials[(tile, split)] = timeit(lambda: run(tile, split), a.reps)
                except Exception as e:  # noqa: BLE001 - workspace or shape limits
                    trials[(tile, split)] = float("inf")
        c["C"].copy_(C_save)
        if not trials:
            trials[(AUTO, 0)] = t_auto
        best = min(trials, key=trials.get)
        n = len(cs)
        tot_auto += t_auto * n
        tot_lib += t_lib * n
        tot_best += trials[best] * n
        Ash, Bsh, Csh = key[0], key[2], key[4]
        M, K = Ash[-2], Ash[-1]
        N = Bsh[-1]
        bt = max(len(Ash) == 3 and Ash[0] or 1, len(Csh) == 3 and Csh[0] or 1, len(Bsh) == 3 and Bsh[0] or 1)
        fl = 2.0 * M * N * K * bt
        row = {"M": M, "N": N, "K": K, "batch": bt, "A_stride": key[1], "B_stride": key[3], "calls": n,
               "auto_us": t_auto, "best": [TILES[best[0]], best[1]], "best_us": trials[best],
               "auto_tflops": fl / t_auto / 1e6, "best_tflops": fl / trials[best] / 1e6,
               "trials": {f"{TILES[k[0]]}/s{k[1]}": v for k, v in trials.items()}}
        res.append(row)
        print(f"M{M:6d} N{N:5d} K{K:6d} b{bt} x{n:2d} A{key[1]} B{key[3]}: auto {t_auto:7.1f}us "
              f"({row['auto_tflops']:5.1f} TF)  best {TILES[best[0]]}/s{best[1]} {trials[best]:7.1f}us "
              f"({row['best_tflops']:5.1f} TF)  torch.matmul {t_lib:7.1f}us ({fl / t_lib / 1e6:5.1f} TF){extra}", flush=True)
    print(f"step gemm total: auto {tot_auto:.0f} us, best {tot_best:.0f} us, torch.matmul {tot_lib:.0f} us"
          + (f", flag {a.flag}: {globals()['_tot_flag'][0]:.0f} us" if a.flag else ""))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
