"""Training-step throughput of the ALIGNN hot path on MI355X (BASELINE.json metric).

One step = the per-batch body of ``train_epoch_hetero`` (scripts/train.py:639-699) on a batch of
B synthetic MP-like graphs (60 atoms / 720 bonds / 7,920 triplets each), D=256, H=4,
L=4, dropout 0.15, feature jitter 0.1: forward, hetero NLL, backward, clip_grad_norm_(5), AdamW.
Inputs are collated and resident in HBM before the timed region (CSR built once per batch).

Multi-GPU: one process per GPU (torch.distributed.run, started by bench.py itself for --gpus N);
each rank trains on its own batch of B graphs (weak scaling) and the gradients are averaged over the
flat gradient buffer (13.2 MB fp32) per step in two buckets, the first (the conv blocks, 10.4 MB)
all_reduced while the backward's tail runs — the data-parallel exchange of SURVEY §8e.

Prints one JSON line (rank 0).  Also reports the dominant kernel's roofline (HIP events around
its launches inside the timed region) and the oracle's CPU throughput on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gnn-elasticity-predictor_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "graphs/sec fwd+bwd (ALIGNN, ~60-atom MP crystals) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def survey_bytes_per_graph(s: int, D: int = 256, L: int = 4, N: int = 60, E: int = 720, T: int = 7920,
                           Fn: int = 206, Fe: int = 36, Fa: int = 11) -> float:
    """SURVEY §8d's compulsory HBM bytes per MP-like graph (ideal fusion, s bytes per activation):
    inp = 4(N Fn + E Fe + T Fa + 291) + 4(2E + 2T + N); fwd_l = s(TD + 3ED + 2ND);
    bwd_l = 2 fwd_l + 8TD; bytes = inp + L(fwd_l + bwd_l).  190.8 MB at s = 4, 128.1 MB at s = 2."""
    inp = 4 * (N * Fn + E * Fe + T * Fa + 291) + 4 * (2 * E + 2 * T + N)
    fwd_l = s * (T * D + 3 * E * D + 2 * N * D)
    return float(inp + L * (fwd_l + 2 * fwd_l + 8 * T * D))
FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32-input MFMA dense peak
BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 dense MFMA peak (no sparsity)
PROBE_STEPS = 3            # untimed replays the dominant-kernel ranking sums over
C1_WARM, C1_REPS = 10, 50   # config C1 forward timing (median of 50 after 10)
CPU_BUDGET_S = 40.0        # CPU baseline: time-boxed sample (cpu_baseline)
SERIAL_STEPS = 3           # serialised replays after the timed region (the dominant kernel's own duration)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="GPUs (= ranks) of one node.  Without a torch.distributed launcher in the environment "
                        "(no WORLD_SIZE) and N > 1, bench.py starts the N rank processes itself "
                        "(torch.distributed.run, 127.0.0.1) before anything touches the GPU")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend of a multi-rank run (nccl = RCCL over xGMI; gloo only to rehearse "
                        "the multi-rank path where RCCL cannot run, e.g. several ranks on one GPU)")
    p.add_argument("--share-device", action="store_true",
                   help="every rank on cuda:0 (with --dist-backend gloo: a multi-rank rehearsal on a one-GPU box)")
    p.add_argument("--dry-run", action="store_true",
                   help="no GPU: every rank runs only the data-parallel exchange (gloo all_reduce of a flat "
                        "gradient of the model's size) — a CPU rehearsal of the rank plumbing")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=32, help="graphs per GPU (BASELINE config 2: 32)")
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--layers", type=int, default=4)
    p.add_argument("--heads", type=int, default=4)
    p.add_argument("--dropout", type=float, default=0.15)
    p.add_argument("--lg-offset", default="num_nodes", choices=["num_nodes", "num_edges"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-steps", type=int, default=5, help="minimum CPU-baseline steps (time-boxed beyond)")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the secondary lines of the default one-GPU run (corrected wiring, config C3)")
    p.add_argument("--roofline-parts", default="probe,stamps,serial",
                   help="diagnostics: which parts of the roofline measurement run (probe = the dominant-kernel "
                        "probe capture, stamps = timestamps in the timed capture, serial = serialised replays)")
    p.add_argument("--secondaries", default="cw,c1,c3,c5,c4,var",
                   help="which secondary lines the default one-GPU run measures (diagnostics): cw = corrected "
                        "wiring, c1 = C1 forward, c3 = C3 step, c5 = C5 loop (needs c3), c4 = C4 predict, "
                        "var = the e2e_variable loop")
    p.add_argument("--dump-probes", default="", help="write the per-op probe summary (JSON) to this path")
    p.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                   help="GEMM arithmetic: fp32 (BASELINE config 2, the default) or bf16 matrix-core inputs with "
                        "fp32 accumulation (config 3's autocast precision; a secondary line, never the fp32 number)")
    p.add_argument("--e2e", type=int, default=10000, metavar="GRAPHS",
                   help="also time the end-to-end loop over an HBM-resident dataset of this many graphs per rank "
                        "(config C5's ~10k graphs; 0 = off): device collate of a random batch + CSR/compaction + "
                        "step, at the headline config and (one GPU) at config C5's B=256 bf16 (SURVEY §8d's "
                        "'including collate' number; separate fields, never value)")
    p.add_argument("--launch", choices=["eager", "plan", "graph"], default="plan",
                   help="eager: Python issues every launch; plan: the step is recorded once as a native launch "
                        "plan and re-issued from C++ (plan.hip; the roofline probe is a pair of plan timestamps "
                        "in every replay); graph: ROCm HIP graphs of the same capture")
    p.add_argument("--graph", action="store_true", help="alias of --launch graph")
    p.add_argument("--ensemble", type=int, default=0, metavar="MEMBERS",
                   help="config C4: train an ensemble of this many members instead (member i on rank i %% world, "
                        "seed +1007 i, fold i %% 5 — train.py:2052-2095 — no per-step communication; several "
                        "members on one GPU run concurrently on their own streams), B = --batch graphs each; then "
                        "one gather of every member's heads on an eval batch to rank 0 for the moment mix")
    p.add_argument("--seed", type=int, default=42, help="base seed of the ensemble members (train.py --seed)")
    p.add_argument("--set", action="append", default=[], metavar="KEY=VAL",
                   help="engine option of this run's model (engine.<attr>=0/1|N), trainer optimizer (optimizer=hip) "
                        "or stream priorities (loader_priority / main_priority / loader_dedicated); repeatable — for measuring "
                        "opt-in paths")
    return p.parse_args()


def apply_settings(args, model):
    """--set KEY=VAL: per-model engine options (engine.<attr>, instance state of this model's engine —
    nothing process-global is changed) and run options; returns the trainer kwargs."""
    kw = {}
    for item in args.set:
        k, v = item.split("=", 1)
        if k.startswith("engine."):
            attr = k.split(".", 1)[1]
            if not hasattr(model._engine, attr):
                raise ValueError(f"unknown engine option {attr}")
            cur = getattr(model._engine, attr)
            if isinstance(cur, str):
                setattr(model._engine, attr, v)
            else:
                setattr(model._engine, attr,
                        int(v) if (isinstance(cur, int) and not isinstance(cur, bool)) else bool(int(v)))
        elif k == "optimizer":
            kw["optimizer"] = v
        elif k == "loader_priority":
            args.loader_priority = int(v)
        elif k == "loader_dedicated":
            args.loader_dedicated = int(v)
        elif k == "main_priority":
            args.main_priority = int(v)
        elif k == "stream_priority":   # the engine's side / aux streams (ops.STREAM_PRIORITY)
            from alignn_mi355x import ops
            ops.STREAM_PRIORITY = int(v)
        elif k == "prefetch":          # e2e loops: batches prepared ahead on the loader stream
            args.prefetch = int(v)
        else:
            raise ValueError(f"unknown --set key {k}")
    return kw


def _cpu_threads() -> int:
    """Host threads for the CPU baseline: the CPUs this process may use.  On the GPU box the job's
    CPU share is set by OMP_NUM_THREADS (16 per GPU) while os.cpu_count() reports the whole machine;
    more threads than the share would oversubscribe it."""
    env = os.environ.get("ALIGNN_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(args, B):
    """The oracle (PyTorch-CPU restatement of the reference's path, fp32) on a bounded sample of the
    same workload: full fwd + NLL + bwd + clip + AdamW steps on the same synthetic graphs, protocol
    of SURVEY §8d (all usable host threads, per-step median after warm-up)."""
    from oracle import model_ref
    from oracle.pyg_ref import RefData, collate

    from alignn_mi355x.synthetic import TARGET_LOG_MEANS, TARGET_LOG_STDS, mp_like_graph
    import alignn_mi355x as A

    threads = _cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, args.hidden, args.layers, args.heads,
                                                          0.0), 2)
        st = {k: v.detach().clone() for k, v in model.state_dict().items()}
        gs = [mp_like_graph(g) for g in range(B)]
        b = collate([RefData(**{k: getattr(d, k) for k in d.keys()}) for d in gs], lg_offset=args.lg_offset)
        # SURVEY §8d asks for the median of 50 steps after 10 warm-ups; at ~4 s per step on the host that
        # is minutes, so the sample is time-boxed: 2 warm-up steps, then steps until CPU_BUDGET_S have
        # passed (at least args.cpu_steps), reported as p10 / p50 / p90 with the step count
        for _ in range(2):
            model_ref.train_step(st, b, args.heads, TARGET_LOG_MEANS, TARGET_LOG_STDS, steps=1)
        times = []
        t_start = time.perf_counter()
        while len(times) < args.cpu_steps or (time.perf_counter() - t_start < CPU_BUDGET_S and len(times) < 50):
            t0 = time.perf_counter()
            model_ref.train_step(st, b, args.heads, TARGET_LOG_MEANS, TARGET_LOG_STDS, steps=1)
            times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    times.sort()
    q = lambda f: times[min(len(times) - 1, int(f * len(times)))]  # noqa: E731
    med = q(0.5)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(B / med, 3), "unit": "graphs/s", "cores": threads, "kind": "port",
            "p10_p50_p90_graphs_per_s": [round(B / q(0.9), 3), round(B / med, 3), round(B / q(0.1), 3)],
            "steps_timed": len(times),
            "sample": f"median of {len(times)} steps x {B} graphs (fp32 fwd+NLL+bwd+clip+AdamW, dropout 0) after "
                      f"2 warm-up steps, time-boxed to {CPU_BUDGET_S:.0f} s (p10/p50/p90 beside it), "
                      f"torch.set_num_threads({threads}) (the job's CPU share; os.cpu_count() = {os.cpu_count()}); "
                      f"{cpu_model}"}


def c1_forward(args, dev, lender=None):
    """Config C1: one graph, forward only, fp32 — (1a) the reference's smoke shape
    (tests/smoke.py:106-145: node/edge/angle dims 6/8/7, hidden 32, 1 layer, 1 head) and (1b) one
    MP-like graph at L = 1 (D = 256, H = 4).  The reference's CPU path (the oracle, all of the job's
    host threads) and the engine on the GPU (model(batch) in eval mode, synchronised per call: the
    latency of one forward), each the median of C1_REPS calls after C1_WARM warm-up calls."""
    from oracle import model_ref
    from oracle.pyg_ref import RefData, collate

    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_graph, si2_smoke_graph

    threads = _cpu_threads()
    prev = torch.get_num_threads()
    out = {}
    shapes = {"c1a_smoke_shape": ((6, 8, 7, 289, 2, 32, 1, 1, 0.0), lambda: si2_smoke_graph(0), 1),
              "c1b_mp_like_L1": ((206, 36, 11, 289, 2, args.hidden, 1, args.heads, 0.0), lambda: mp_like_graph(0),
                                 args.heads)}
    for name, (cfg, graph, heads) in shapes.items():
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(*cfg), 2).eval()
        if lender is not None:   # no streams of its own beside the idle headline trainer's (see measure)
            model._engine.ctx.borrow_streams(lender.model._engine.ctx)
        st = {k: v.detach().clone() for k, v in model.state_dict().items()}
        g = graph()
        ref = collate([RefData(**{k: getattr(g, k) for k in g.keys()})], lg_offset=args.lg_offset)

        def cpu_fwd():
            with torch.no_grad():
                model_ref.hetero_forward(st, ref, heads)

        torch.set_num_threads(threads)
        try:
            t_cpu = _median_time(cpu_fwd, C1_WARM, C1_REPS, sync=False)
        finally:
            torch.set_num_threads(prev)
        model.to(dev)
        b = A.Batch.from_data_list([g]).to(dev)

        def gpu_fwd():
            with torch.no_grad():
                model(b)

        t_gpu = _median_time(gpu_fwd, C1_WARM, C1_REPS, sync=True)
        out[name] = {"graph": {"atoms": int(g.x.size(0)), "bonds": int(g.edge_index.size(1)),
                               "triplets": int(g.lg_edge_index.size(1))},
                     "model": dict(zip(("node_dim", "edge_dim", "angle_dim", "global_dim", "targets", "hidden",
                                        "layers", "heads"), cfg[:8])),
                     "cpu_ms": round(t_cpu * 1e3, 3), "cpu_threads": threads,
                     "gpu_ms": round(t_gpu * 1e3, 3), "speedup": round(t_cpu / t_gpu, 1)}
        del model, b
    out["protocol"] = (f"forward only, fp32, eval mode; median of {C1_REPS} calls after {C1_WARM} warm-up; the GPU "
                       f"figure is one model(batch) call synchronised (host launch latency included; the call replays "
                       f"the recorded forward from the second call on, alignn_mi355x/infer.py)")
    return out


def _median_time(fn, warm, reps, sync):
    for _ in range(warm):
        fn()
    if sync:
        torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def ensemble_predict(args, dev, members=5, B=256):
    """predict.ensemble_predict / ensemble_collect (predict.py:582-653, train.py:849-904) at config C4's
    shape on one GPU: `members` models at B graphs, bf16 (the reference predicts under autocast),
    EnsemblePredictor.predict_batch — every member's forward on its own stream, the moment mix and the
    log-normal conversion — timed per batch with the forwards as replayed plans (infer.py) and eager."""
    import alignn_mi355x as A
    from alignn_mi355x import infer
    from alignn_mi355x.ensemble import EnsemblePredictor
    from alignn_mi355x.synthetic import mp_like_batch
    models = []
    for i in range(members):
        torch.manual_seed(1000 + i)
        m = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, args.hidden, args.layers, args.heads,
                                                      args.dropout), 2).to(dev).eval()
        models.append(m.set_precision("bf16"))
    batches = [mp_like_batch(B, first=B * i).to(dev) for i in range(2)]
    ep = EnsemblePredictor(models)
    out = {"members": members, "batch": B, "precision": "bf16"}
    it = {"k": 0}

    def call():
        r = ep.predict_batch(batches[it["k"] % 2])   # alternating batches: every plan call re-binds
        it["k"] += 1
        return r

    for name, enabled in (("plan", True), ("eager", False)):
        infer.ENABLED = enabled
        try:
            t = _median_time(call, 4, 20, sync=True)
        finally:
            infer.ENABLED = True
        out[f"{name}_ms_per_batch"] = round(t * 1e3, 3)
        out[f"{name}_graphs_per_s"] = round(B / t, 1)
    for m in models:
        infer.release(m)
    out["protocol"] = ("median of 20 predict_batch calls after 4 warm-up, alternating two batches of the same "
                       "signature; synchronised per call")
    return out


def build_store(args, dev, rank):
    """This rank's shard of an HBM-resident dataset of args.e2e synthetic MP-like graphs
    (store.GraphStore; config C5's ~10k-graph dataset split over the data-parallel ranks), built
    once and shared by the end-to-end loops."""
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_graph

    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    t0 = time.perf_counter()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    per = (args.e2e + world - 1) // world
    first = rank * per
    n = max(1, min(per, args.e2e - first))
    store = GraphStore.from_data_list([Data(**{k: getattr(mp_like_graph(first + g), k) for k in keys})
                                       for g in range(n)], dev)
    torch.cuda.synchronize()
    return store, time.perf_counter() - t0


def end_to_end(args, store, t_build, trainer, B, dev, rank, world, capacity=None):
    """The reference's training loop (train.py:639-711) over a dataset resident in HBM: per step a
    random batch is collated on the device and its CSR lists / line-graph compaction / schedules are
    built on a loader stream (engine.prepare_batch) while the previous step runs; the step re-binds
    the captured plan to it (FusedTrainer._rebind: copies into the captured batch's buffers) and
    replays.  Timed like the headline: barrier + synchronize on both sides, max over ranks."""
    import numpy as np
    from alignn_mi355x import ops as _ops
    from alignn_mi355x.dp import max_over_ranks
    from alignn_mi355x.engine import prepare_batch

    rng = np.random.default_rng(1234 + rank)
    # The loader stream: a pooled stream at the step's priority (high).  A dedicated hardware queue for
    # it (round 4) stopped paying once the step used three streams: the process's GPU_MAX_HW_QUEUES = 4
    # queues are then shared, and the dedicated queue pushed the other loops' streams together — with
    # the secondaries' trainers alive the B = 32 loop fell to 71 % of the bare step (BENCH_r05); without
    # them every placement gives 92 %, and the padded loop after a dedicated queue had been created
    # lost a third (gpurun_out r6a: B = 32 e2e 9,930-10,040 graphs/s for dedicated / pooled / pooled at
    # high priority / prefetch 2; e2e_variable 7,200 after the dedicated queue vs 11,400 without).
    # (--set loader_priority=0 / loader_dedicated=1 / main_priority=0 keep the earlier placements.)
    # Round 6: the remaining loss (the loop at 67-71 % of the bare step whenever anything had been
    # captured before it — the roofline probe, a secondary's trainer) was a new pooled warm-up stream
    # per capture, which moved this stream's hardware-queue assignment onto one of the step's; every
    # capture now warms up on one process-wide stream (ops.warmup_stream): 7,400 -> 9,820 graphs/s
    # with the probe (gpurun_out r6y, r6ad).
    prio = getattr(args, "loader_priority", None)
    if prio is None:
        prio = args.main_priority if args.main_priority else (-1 if B >= 128 else 0)
    dedicated = prio == 0 and bool(int(getattr(args, "loader_dedicated", 0)))
    loader = None
    if dedicated:
        try:
            loader = _ops.dedicated_stream(dev)
        except RuntimeError as e:   # reported in the line; the loop still runs on a pooled stream
            print(f"[bench] dedicated loader queue unavailable ({e}); pooled stream", file=sys.stderr)
            dedicated = False
    if loader is None:
        loader = torch.cuda.Stream(device=dev, priority=prio)

    def make():
        with torch.cuda.stream(loader):
            b = store.collate(rng.choice(store.num_graphs, size=B, replace=False), lg_offset=args.lg_offset,
                              capacity=capacity)
        prepare_batch(b, loader)
        return b

    r0, m0 = trainer.rebinds, trainer.rebind_misses
    depth = max(1, int(getattr(args, "prefetch", 1) or 1))   # batches prepared ahead
    ahead = [make() for _ in range(depth)]
    # (at least 20 untimed steps: the first loop over a fresh store measured 10-30 % slow after 5)
    for i in range(max(args.warmup, 20)):
        cur = ahead.pop(0)
        trainer.step(cur, seed=7919 * rank + i)
        ahead.append(make())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    host_step = host_make = 0.0
    t0 = time.perf_counter()
    for i in range(args.steps):
        cur = ahead.pop(0)
        ta = time.perf_counter()
        trainer.step(cur, seed=7919 * rank + max(args.warmup, 20) + i)
        tb = time.perf_counter()
        ahead.append(make())
        host_step += tb - ta
        host_make += time.perf_counter() - tb
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = max_over_ranks(dt, dev)
    out = {"value": round(B * world * args.steps / dt, 2), "unit": "graphs/s",
           "ms_per_step": round(dt / args.steps * 1e3, 3), "batch": B, "dataset_graphs": args.e2e,
           "dataset_graphs_per_rank": store.num_graphs,
           "store_build_s": round(t_build, 1), "replayed_steps": trainer.rebinds - r0,
           "host_ms_per_step": {"rebind_and_replay": round(host_step / args.steps * 1e3, 3),
                                "collate_and_prepare": round(host_make / args.steps * 1e3, 3)},
           "eager_steps": trainer.rebind_misses - m0,
           "stream_priorities": {"step": args.main_priority, "loader": prio, "prefetch": depth,
                                 "loader_queue": "dedicated" if dedicated else "pooled"},
           "signature": ("every batch padded to one capacity (store.BatchCapacity)" if capacity is not None else
                         "fixed: every synthetic graph has 60 atoms, so every batch has the captured signature "
                         "(best case; see e2e_variable for variable-size graphs)"),
           "includes": "device collate of a random batch + CSR/compaction/schedules (loader stream) + "
                       "fwd/NLL/bwd/clip/AdamW (captured plan re-bound to the batch)"}
    return out


def build_variable_store(args, dev, rank):
    """This rank's shard of a dataset of variable-size MP-like graphs (8-60 atoms, 2-6 neighbour
    shells: synthetic.variable_mp_like_graph), built once."""
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import variable_mp_like_graph

    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    t0 = time.perf_counter()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    per = (args.e2e + world - 1) // world
    first = rank * per
    n = max(1, min(per, args.e2e - first))
    store = GraphStore.from_data_list([Data(**{k: getattr(variable_mp_like_graph(first + g), k) for k in keys})
                                       for g in range(n)], dev)
    torch.cuda.synchronize()
    return store, time.perf_counter() - t0


def end_to_end_variable(args, dev, rank, world, B):
    """The reference's loop over real-crystal-like data: graphs of variable size, every batch padded to
    one capacity by a ghost graph (store.BatchCapacity) so that the plan captured once is re-bound to
    every batch.  value = real graphs per second."""
    import alignn_mi355x as A
    import numpy as np
    from alignn_mi355x.dp import GradBuckets
    from alignn_mi355x.layout import bucket_split
    store, t_build = build_variable_store(args, dev, rank)
    cap = store.capacity(B, args.lg_offset)
    torch.manual_seed(1234)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, args.hidden, args.layers, args.heads,
                                                      args.dropout), 2).to(dev)
    trainer = A.FusedTrainer(model, precision=args.precision)
    if world > 1:
        trainer.grad_buckets = GradBuckets(trainer.st.grad, bucket_split(model.config, True), world)
    rng = np.random.default_rng(99)
    first = next(i for i in (rng.choice(store.num_graphs, size=B, replace=False) for _ in range(1000))
                 if store.fits(i, cap, args.lg_offset) is not None)
    trainer.capture(store.collate(first, lg_offset=args.lg_offset, capacity=cap))
    sizes = [store.batch_sizes(np.random.default_rng(s).choice(store.num_graphs, size=B, replace=False),
                               args.lg_offset)["nodes"] for s in range(64)]
    r = end_to_end(args, store, t_build, trainer, B, dev, rank, world, capacity=cap)
    r["capacity"] = {"graphs": cap.graphs, "nodes": cap.nodes, "edges": cap.edges, "triplets": cap.triplets,
                     "active_bonds": cap.active}
    r["mean_real_atoms_per_batch"] = round(float(np.mean(sizes)), 1)
    r["real_atom_fraction_of_capacity"] = round(float(np.mean(sizes)) / cap.nodes, 3)
    trainer.release_capture()
    return r


def pmc_traffic(kernel_key):
    """HBM bytes per launch of ``kernel_key`` from the committed PMC passes (profiles/pmc_dominant.json:
    FETCH_SIZE x2 + WRITE_SIZE, tools/pmc_traffic.py), or None when that kernel/shape was not counted."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_dominant.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(kernel_key)
    except (OSError, ValueError):
        return None
    return None if rec is None else rec["traffic_bytes"]


def _roofline(summ, dominant, mfma_peak, probe_src):
    """The dominant kernel against the roof that binds it: a GEMM is MFMA-bound when its arithmetic
    intensity (algorithmic flops / bytes: A, B and C once) times the HBM peak exceeds the matrix-core
    peak, HBM-bound otherwise (the bf16 products over every bond: 64 flop/B x 8 TB/s < 2.5 PF/s);
    the attention kernels are HBM-bound."""
    s = summ[dominant]
    avg_s = s["avg_ms"] / 1e3
    flops, nbytes = s["flops_per_launch"], s.get("bytes_per_launch", 0.0)
    if flops > 0 and nbytes > 0 and flops / nbytes * HBM_PEAK_GBS / 1e3 < mfma_peak:
        flops = 0.0   # below the ridge point: report it against HBM
    if flops > 0:
        ach = s["flops_per_launch"] / avg_s / 1e12
        return {"bound": "mfma", "achieved": round(ach, 2), "peak": mfma_peak, "unit": "TFLOP/s",
                "frac": round(ach / mfma_peak, 4), "traffic": pmc_traffic(dominant), "kernel": dominant,
                "avg_us": round(s["avg_ms"] * 1e3, 2), "launches": s["count"],
                "flops_per_launch": s["flops_per_launch"], "timing": probe_src}
    ach = s["bytes_per_launch"] / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(dominant), "kernel": dominant,
            "avg_us": round(s["avg_ms"] * 1e3, 2), "launches": s["count"],
            "bytes_per_launch": s["bytes_per_launch"], "timing": probe_src}


def measure(args, dev, rank, world, B, lg_offset, precision, steps, warmup, roofline=True, streams_of=None):
    """Builds the model, trainer and a resident batch of B graphs, picks the dominant kernel (one
    untimed eager probe step), captures the step, runs `warmup` steps and times exactly `steps`
    (barrier + synchronize on both sides, max over ranks).  Returns the numbers and the trainer.
    ``streams_of``: an idle trainer whose side / aux streams this one uses (ExecContext.borrow_streams)."""
    import alignn_mi355x as A
    from alignn_mi355x import profiling
    from alignn_mi355x.dp import GradBuckets, max_over_ranks, rank_graphs
    from alignn_mi355x.layout import bucket_split
    from alignn_mi355x.synthetic import mp_like_batch

    torch.manual_seed(1234)  # identical initial weights on every rank
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, args.hidden, args.layers, args.heads,
                                                      args.dropout), 2).to(dev)
    if streams_of is not None:
        model._engine.ctx.borrow_streams(streams_of.model._engine.ctx)
    trainer = A.FusedTrainer(model, precision=precision, **apply_settings(args, model))
    mfma_peak = BF16_MFMA_TFLOPS if precision == "bf16" else FP32_MFMA_TFLOPS
    batch = mp_like_batch(B, first=rank_graphs(B, rank).start, lg_offset=lg_offset).to(dev)
    if world > 1:
        # the DP exchange: the flat gradient's mean in two buckets, the first beside the backward's tail
        trainer.grad_buckets = GradBuckets(trainer.st.grad, bucket_split(model.config, True), world)

    def step(i):
        trainer.step(batch, seed=1000003 * rank + i)

    # pick the dominant kernel: the probed family (GEMM shape / attention launch) with the largest
    # total device time summed over PROBE_STEPS untimed steps.  With native plans the probe is a
    # separate capture whose every probed launch is bracketed by plan timestamps, replayed SERIALISED
    # (every launch on one stream, alignn_plan_replay_serial): each kernel's own duration, as a PMC
    # pass runs it.  In-step timestamps of a multi-stream replay include the time a launch queues
    # behind the other streams' kernels (round 4, C3: the atom-graph backward at 749 us in-step
    # against 279 us in a rocprofv3 trace and 202 us under the counters), so ranking on them measured
    # overlap, not kernels.
    dominant, step_work = None, None
    parts = set(getattr(args, "roofline_parts", "probe,stamps,serial").split(","))
    if roofline and "probe" not in parts:
        dominant = "gemm_f32 M23040 N256 K256 b1" if B == 32 else None
    if roofline and "probe" in parts:
        totals, summ = {}, {}
        plan_probe = args.launch == "plan"
        if plan_probe:
            profiling.enable(None)
            trainer.capture(batch, mode="plan")
            profiling.disable()
        else:
            step(0)
            torch.cuda.synchronize()
        trainer.serial_replay = plan_probe
        for i in range(PROBE_STEPS):
            if not plan_probe:
                profiling.enable(None)
            step(1 + i)
            torch.cuda.synchronize()
            summ = profiling.summary()
            if not plan_probe:
                profiling.disable()
            for k, v in summ.items():
                totals[k] = totals.get(k, 0.0) + v["total_ms"]
        trainer.serial_replay = False
        if plan_probe:
            trainer.release_capture()
        profiling.clear()
        dominant = max(totals, key=lambda k: (totals[k], k))
        # whole-step algorithmic work of this formulation (one probe step): GEMM flops, attention bytes
        step_work = {"gemm_gflop": sum(v["flops_per_launch"] * v["count"] for v in summ.values()) / 1e9,
                     "tconv_gbyte": sum(v["bytes_per_launch"] * v["count"] for k, v in summ.items()
                                        if k.startswith("tconv")) / 1e9}
        if args.dump_probes and rank == 0 and (B, lg_offset, precision) == (args.batch, args.lg_offset,
                                                                             args.precision):
            with open(args.dump_probes, "w") as f:
                json.dump({k: dict(summ[k], total_ms_probe_steps=totals[k]) for k in
                           sorted(summ, key=lambda k: -totals[k])}, f, indent=1)

    # captured step: in a plan the dominant kernel's launches are bracketed by plan timestamps, so
    # every replay re-times them; the timed region's last replay is read back afterwards
    launch_mode, probe_in_graph = "eager", False
    if args.launch != "eager":
        mode = args.launch
        # ROCm refuses external event nodes in a captured graph: graph mode probes eagerly after
        # the timed region; a plan carries the probes as timestamps
        if dominant is not None and mode == "plan" and "stamps" in parts:
            profiling.enable(dominant)
        trainer.capture(batch, mode=mode)
        probe_in_graph = dominant is not None and mode == "plan" and "stamps" in parts
        launch_mode = "native_plan" if mode == "plan" else "hip_graph"
        profiling.disable()

    for i in range(warmup):
        step(2 + i)
    torch.cuda.synchronize()

    if launch_mode == "eager" and dominant is not None:
        profiling.enable(dominant)   # events around each launch of the dominant kernel, timed region
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(2 + warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    profiling.disable()
    if world > 1:
        dt = max_over_ranks(dt, dev)
    if probe_in_graph:
        try:  # the plan timestamps hold the last replay's times
            probe_in_graph = profiling.summary()[dominant]["avg_ms"] > 0
        except Exception as e:  # noqa: BLE001
            print(f"[bench] plan probe timing unavailable ({e}); probing eagerly", file=sys.stderr)
            probe_in_graph = False
    if dominant is not None and launch_mode != "eager" and not probe_in_graph and "stamps" in parts:
        # fallback: time the dominant kernel in two extra eager steps after the timed region
        saved = trainer._graph
        trainer._graph = None
        profiling.enable(dominant)
        profiling.clear()
        for i in range(2):
            step(10**6 + i)
        torch.cuda.synchronize()
        profiling.disable()
        trainer._graph = saved
    probe_src = ("plan timestamps in the replayed step (last timed replay)" if (probe_in_graph and launch_mode == "native_plan") else
                 "hip events in the captured step (last timed replay)" if probe_in_graph else
                 "hip events around each launch, timed region" if launch_mode == "eager" else
                 "hip events, 2 eager steps after the timed region")
    value = B * world * steps / dt
    summ = profiling.summary() if dominant is not None else {}
    in_step = summ.get(dominant)
    if probe_in_graph and launch_mode == "native_plan" and "serial" in parts:
        # the kernel's own duration: the same plan replayed serialised (after the timed region); the
        # in-step figure (last timed replay) stays beside it
        trainer.serial_replay = True
        for i in range(SERIAL_STEPS):
            step(2 * 10**6 + i)
        torch.cuda.synchronize()
        trainer.serial_replay = False
        summ = profiling.summary()
        probe_src = f"plan timestamps, plan replayed serialised on one stream (last of {SERIAL_STEPS} replays after the timed region)"
    roof = _roofline(summ, dominant, mfma_peak, probe_src) if (dominant is not None and dominant in summ) else None
    if roof is not None and in_step is not None:
        roof["avg_us_in_step"] = round(in_step["avg_ms"] * 1e3, 2)
    step_roof = None if step_work is None else {
        # whole-step view: this formulation's GEMM flops and attention bytes per graph
        # and the fraction of the MFMA / HBM peaks they imply at the measured rate
        "gemm_gflop_per_graph": round(step_work["gemm_gflop"] / B, 4),
        "mfma_frac": round(step_work["gemm_gflop"] / B * (value / world) / (mfma_peak * 1e3), 4),
        "tconv_mbyte_per_graph": round(step_work["tconv_gbyte"] * 1e3 / B, 2),
        "hbm_frac": round(step_work["tconv_gbyte"] / B * value / world / HBM_PEAK_GBS, 4),
        # the north-star figure for bf16: the survey's per-graph bytes at the measured rate
        "survey_mbyte_per_graph": round(survey_bytes_per_graph(2 if precision == "bf16" else 4) / 1e6, 2),
        "survey_hbm_frac": round(survey_bytes_per_graph(2 if precision == "bf16" else 4) / 1e9 * value / world
                                 / HBM_PEAK_GBS, 4)}
    return {"value": value, "dt": dt, "ms_per_step": dt / steps * 1e3, "launch": launch_mode, "roofline": roof,
            "step_roofline": step_roof, "trainer": trainer, "batch": batch}


def ensemble_bench(args, dev, rank, world):
    """Config C4: ensemble training sharded member-per-rank.  The reference trains its
    members one after the other (train.py:2052-2095); here every rank trains its members
    (dp.members_of_rank) at the same time — each member a captured step on its own stream — with no
    communication until the final gather of the members' heads for the moment mix.  Timed like the
    headline (barrier + synchronize, max over ranks); value = members x B x steps / time."""
    import alignn_mi355x as A
    from alignn_mi355x import dp
    from alignn_mi355x.ensemble import EnsemblePredictor, EnsembleTrainer, ShardedEnsemble
    from alignn_mi355x.synthetic import ensemble_member_batch, mp_like_batch

    M, B = args.ensemble, args.batch

    def build():
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, args.hidden, args.layers, args.heads,
                                                          args.dropout), 2).to(dev)
        apply_settings(args, model)
        return model

    # the member's own graphs (fold i % 5 of the dataset, train.py:2054): a disjoint synthetic slice
    ens = EnsembleTrainer(M, build, lambda i, fold: ensemble_member_batch(B, i, fold, args.lg_offset).to(dev),
                          world=world, rank=rank, seed=args.seed, precision=args.precision)
    mine = ens.ids
    step = ens.step

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = dp.max_over_ranks(dt, dev)
    # the members' eval pass: heads of every member on one batch, gathered to rank 0, moment mix
    ens.release()
    models = ens.models()
    for model in models:
        model.eval()
    eval_batch = mp_like_batch(B, first=900000, lg_offset=args.lg_offset).to(dev)
    t1 = time.perf_counter()
    if world > 1:
        mixed = ShardedEnsemble(models, M, hidden=args.hidden).predict_batch(eval_batch)
    else:
        mixed = EnsemblePredictor(models).predict_batch(eval_batch)
    torch.cuda.synchronize()
    t_eval = time.perf_counter() - t1
    ok = None if mixed is None else bool(torch.isfinite(mixed["mean_z"]).all() and torch.isfinite(mixed["std_z"]).all())
    return {"value": M * B * args.steps / dt, "dt": dt, "ms_per_step": dt / args.steps * 1e3,
            "members_per_rank": len(mine), "eval_ms": round(t_eval * 1e3, 2), "eval_finite": ok}


def _release(r):
    tr = r.pop("trainer", None)
    r.pop("batch", None)
    if tr is not None:
        tr.release_capture()
    del tr
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _visible_gpus() -> int:
    """Number of GPUs a rank would see, counted in a child interpreter so that this (launcher)
    process never calls into HIP; 0 when the child fails."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else 0
    except (ValueError, IndexError):
        return 0


def launch_ranks(args) -> int:
    """``--gpus N`` run without a launcher: start N ranks with torch.distributed.run on this node
    (rendezvous on 127.0.0.1, a free port), each running this script with the same arguments, and
    return their exit status (non-zero if any rank failed or fewer than N could start).  Nothing
    here touches the GPU: the devices are counted by a child interpreter (_visible_gpus), so no
    process that initialised HIP ever starts another."""
    import socket
    import subprocess
    n = args.gpus
    if not args.dry_run and not args.share_device:
        have = _visible_gpus()
        if have < n:
            print(f"[bench] --gpus {n}: only {have} GPU(s) visible", file=sys.stderr)
            return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only (RCCL across processes)
    env.setdefault("OMP_NUM_THREADS", str(max(1, _cpu_threads() // n)))
    return subprocess.call(cmd, env=env)


def dry_run(args, rank, world):
    """CPU rehearsal of the data-parallel step's exchange: every rank all_reduces (gloo) a flat
    gradient of the model's size each step; timed like the real bench (barrier both sides, max over
    ranks) and reported with the world size the ranks agreed on."""
    from alignn_mi355x.dp import grad_allreduce_hook, max_over_ranks
    from alignn_mi355x.layout import AlignnConfig, offsets
    _, total, _ = offsets(AlignnConfig(206, 36, 11, 289, 2, args.hidden, args.layers, args.heads, 0.0), True)
    grad = torch.full((total,), float(rank + 1))
    hook = grad_allreduce_hook(world)
    for _ in range(args.warmup):
        hook(grad)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        grad.fill_(float(rank + 1))
        hook(grad)
    dist.barrier()
    dt = max_over_ranks(time.perf_counter() - t0, torch.device("cpu"))
    ok = bool(torch.all(grad == (world + 1) / 2.0))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(args.batch * world * args.steps / dt, 2),
                          "unit": "graphs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                          "data": "dry run: no GPU, gloo all_reduce of the flat gradient only",
                          "config": {"workload": "DP exchange rehearsal", "global_batch": args.batch * world,
                                     "parallelism": f"dp{world}", "grad_elems": total, "allreduce_ok": ok}}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    if args.graph:
        args.launch = "graph"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
            return dry_run(args, rank, world)
        raise SystemExit("[bench] --dry-run rehearses the multi-rank exchange: use --gpus N with N > 1")
    if args.share_device:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # every stream of the step at high priority (-1, the highest torch exposes; equal among themselves,
    # so the bare step is unchanged), so that a batch-preparation stream at normal priority takes only
    # what the step leaves idle (end_to_end).  --set main_priority=0 / stream_priority=0: all normal
    settings = dict(x.split("=", 1) for x in args.set)
    args.main_priority = int(settings.get("main_priority", -1))
    from alignn_mi355x import ops as _ops
    _ops.STREAM_PRIORITY = int(settings.get("stream_priority", args.main_priority))
    if args.main_priority:
        hi = torch.cuda.Stream(device=dev, priority=args.main_priority)
        hi.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.set_stream(hi)

    B = args.batch
    if args.ensemble > 0:
        r = ensemble_bench(args, dev, rank, world)
        if rank == 0:
            print(json.dumps({
                "metric": METRIC, "value": round(r["value"], 2), "unit": "graphs/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["ms_per_step"], 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "f32" if args.precision == "fp32" else "bf16-gemm/f32", "data": "synthetic",
                "config": {"workload": f"BASELINE config 4: {args.ensemble}-member ensemble training, B={B} synthetic "
                                       f"MP-like graphs per member per step, full ALIGNN D={args.hidden} H={args.heads} "
                                       f"L={args.layers}, fwd+NLL+bwd+clip+AdamW per member",
                           "global_batch": B * args.ensemble, "parallelism": f"ensemble member-per-rank over {world}",
                           "members_per_rank_0": r["members_per_rank"], "precision": args.precision,
                           "lg_offset": args.lg_offset, "launch": "native_plan (one stream per member)"},
                "ensemble_eval": {"gather_and_mix_ms": r["eval_ms"], "finite": r["eval_finite"]}}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    sec_on = set(args.secondaries.split(","))
    store = None
    if args.e2e > 0 and "store_first" in sec_on:   # diagnostics: the dataset resident before any step
        store, t_build = build_store(args, dev, rank)
    r = measure(args, dev, rank, world, B, args.lg_offset, args.precision, args.steps, args.warmup,
                roofline=not args.no_roofline)

    # secondary lines of the default run (one GPU): the same step with the corrected line-graph
    # wiring (SURVEY §8d "also report num_edges": no compaction, every bond active) and config C3
    # (B = 256, bf16 matrix-core inputs, its own dominant-kernel roofline).  Never `value`.  The
    # pre-collated steps are all measured before the e2e dataset is built, each with at most one other
    # captured trainer alive (the C3 step measured with the dataset resident and after the e2e loops
    # read 8 % low: 16,900 vs 18,400-18,500 graphs/s; the corrected wiring with two other trainers
    # alive 5,100 vs 5,580).
    e2e = None
    if args.e2e > 0 and "e2e_first" in sec_on:
        if store is None:
            store, t_build = build_store(args, dev, rank)
        e2e = end_to_end(args, store, t_build, r["trainer"], B, dev, rank, world)
    secondary, c3 = None, None
    if world == 1 and not args.no_secondary:
        secondary = {}
        sec_steps, sec_warm = max(5, args.steps // 2), max(2, args.warmup // 2)
        if args.lg_offset == "num_nodes" and "cw" in sec_on:
            w = measure(args, dev, rank, world, B, "num_edges", args.precision, sec_steps, sec_warm, roofline=True,
                        streams_of=r["trainer"])
            secondary["corrected_wiring"] = {
                "config": f"B={B}, lg_offset=num_edges (every bond active: no line-graph compaction), {args.precision}",
                "value": round(w["value"], 2), "unit": "graphs/s", "ms_per_step": round(w["ms_per_step"], 3),
                "steps": sec_steps, "roofline": w["roofline"]}
            _release(w)
        if not args.no_cpu_baseline and "c1" in sec_on:
            secondary["c1_forward"] = c1_forward(args, dev, lender=r["trainer"])
        if (B, args.precision) != (256, "bf16") and "c3" in sec_on:
            c3 = measure(args, dev, rank, world, 256, args.lg_offset, "bf16", sec_steps, sec_warm, roofline=True,
                         streams_of=r["trainer"])
            secondary["c3_b256_bf16"] = {
                "config": "BASELINE config 3: B=256 per GPU, bf16 matrix-core inputs (fp32 accumulation, fp32 "
                          f"softmax/LayerNorm), lg_offset={args.lg_offset}",
                "value": round(c3["value"], 2), "unit": "graphs/s", "ms_per_step": round(c3["ms_per_step"], 3),
                "steps": sec_steps, "roofline": c3["roofline"], "step_roofline": c3["step_roofline"]}

    if args.e2e > 0 and store is None:
        store, t_build = build_store(args, dev, rank)
        # The two loops' throughput depends on how their streams share the device's hardware queues
        # (GPU_MAX_HW_QUEUES = 4 here: step main/side/aux + loader + idle streams of the other trainer):
        # whichever loop runs second measured 8-10 % higher in either order (round 4, gpurun_out
        # r4i/r4j/r4k: C5 first 16,560-16,790 vs second 18,570-18,650 graphs/s; B = 32 first 5,760-5,800
        # vs second 8,450-8,610).  C5 (a VERDICT item) runs second.
        if e2e is None:
            e2e = end_to_end(args, store, t_build, r["trainer"], B, dev, rank, world)
        if c3 is not None and "c5" in sec_on:
            # config C5 at N = 1: the B = 256 bf16 step over the ~10k-graph HBM dataset
            secondary["c5_e2e_b256_bf16"] = end_to_end(args, store, t_build, c3["trainer"], 256, dev, rank, world)
    _release(r)
    if c3 is not None:
        _release(c3)
    store = None
    e2e_var = None
    if args.e2e > 0 and "var" in sec_on:
        e2e_var = end_to_end_variable(args, dev, rank, world, B)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    if world == 1 and not args.no_secondary and args.ensemble == 0 and "c4" in sec_on:
        secondary["c4_ensemble_predict_b256"] = ensemble_predict(args, dev)
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, B)
        result = {
            "metric": METRIC, "value": round(r["value"], 2), "unit": "graphs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(r["ms_per_step"], 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "bf16-gemm/f32", "data": "synthetic",
            "config": {"workload": f"B={B} synthetic MP-like graphs per GPU (60 atoms/720 bonds/7920 triplets), "
                                   f"full ALIGNN D={args.hidden} H={args.heads} L={args.layers}, fwd+NLL+bwd+clip+AdamW",
                       "global_batch": B * world, "parallelism": f"dp{world}", "lg_offset": args.lg_offset,
                       "dropout": args.dropout, "launch": r["launch"], "precision": args.precision,
                       **({"dp_exchange": "flat gradient mean in two buckets (conv blocks' parameters reduced "
                                          "beside the backward's tail, then the rest), RCCL all_reduce"}
                          if world > 1 else {}),
                       **({"dist_backend": args.dist_backend + (" (all ranks on cuda:0: rehearsal)" if args.share_device
                                                                 else "")} if world > 1 else {}),
                       **({"settings": args.set} if args.set else {})},
            "roofline": r["roofline"], "cpu_baseline": cpu, "e2e": e2e, "e2e_variable": e2e_var,
            "step_roofline": r["step_roofline"], "secondary": secondary,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
