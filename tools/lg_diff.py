import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "gnn-elasticity-predictor_amd")
from alignn_mi355x import ops
from test_gpu_x_lg3 import DEGREES, _case
DEV = "cuda"
for H in (1, 2, 4):
    for drop in (0.0, 0.15):
        csr, m, t = _case(H, DEGREES["ragged"] + DEGREES["mp_mix"][:20], 90 + H, True)
        n, D = csr.n, 256
        QKV = t["QKVR"][:, :3 * D].contiguous()
        QKV[:, D:3 * D] = QKV[:, D:3 * D].bfloat16().float()
        F = t["F"].bfloat16().float()
        KV16 = ops.cast_bf16(QKV[:, D:3 * D]); F16 = ops.cast_bf16(F)
        outs = {}
        for mode in ("fp32", "bf16"):
            outp, S = torch.empty(n, D, device=DEV), torch.empty(n, H, D, device=DEV)
            sumA, mstat, den = (torch.empty(n, H, device=DEV) for _ in range(3))
            dq = torch.empty(n, D, device=DEV)
            Sz, sigz = torch.empty(n, H, D, device=DEV), torch.empty(n, H, device=DEV)
            dz, al = torch.empty(max(m, 1), H, device=DEV), torch.empty(max(m, 1), H, device=DEV)
            if mode == "fp32":
                ops.tconv_fwd(csr, D, H, QKV, t["U"], t["wbar"], F, None, outp, S, sumA, mstat, den, drop, 5)
                ops.tconv_bwd_dst(csr, D, H, QKV, t["U"], t["Vd"], t["wbar"], F, None, t["dout"], outp, mstat,
                                  den, dq, Sz, sigz, dz, al, None, 0, drop, 5)
            else:
                ops.lg_fwd_bf16(csr, D, H, QKV, KV16, t["U"], t["wbar"], F16, outp, S, sumA, mstat, den, drop, 5)
                ops.lg_bwd_dst_bf16(csr, D, H, QKV, KV16, t["U"], t["Vd"], t["wbar"], F16, t["dout"], outp,
                                    mstat, den, dq, Sz, sigz, dz, al, drop, 5)
            torch.cuda.synchronize()
            outs[mode] = dict(outp=outp, S=S, sumA=sumA, mstat=mstat, den=den, dq=dq, Sz=Sz, sigz=sigz, dz=dz[:m], al=al[:m])
        for k in outs["fp32"]:
            a, b = outs["bf16"][k], outs["fp32"][k]
            if not torch.equal(a, b):
                d = (a - b).abs()
                bad = (d > 0) | (a.isnan() != b.isnan())
                print(H, drop, k, "max abs", float(d.nan_to_num().max()), "ref max", float(b.abs().max()),
                      "n diff", int(bad.sum()), "nan a/b", int(a.isnan().sum()), int(b.isnan().sum()), flush=True)
print("done")
