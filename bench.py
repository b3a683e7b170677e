#!/usr/bin/env python3
"""bench.py -- Gibbs sweeps/s of the MI355X BayesR sampler (BASELINE.json metric).

One step = one full Gibbs sweep (mu, every marker in visit order, hyper-parameters) of
BayesRSamplerV2 on a synthetic cohort resident in HBM (generated on the device, DESIGN.md
"synthetic data spec").  Default workload: BASELINE configs[1] (C2), N = 100,000 individuals
x P = 500,000 f32 genotypes, K = 4 (cva = 1e-4, 1e-3, 1e-2).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|c1]

For N > 1 the driver launches one process per GPU (torch.distributed.run); markers are
column-sharded (contiguous blocks) and the residual is kept coherent by one ncclAllReduce per
sweep inside libbrr (RCCL over xGMI).  torch.distributed is used only with the gloo backend
for the rendezvous, barriers and the max-over-ranks timing -- torch's own HIP runtime is never
initialised in the same process as libbrr (they are different ROCm builds).
Scaling is strong: the same C2 problem is split over the N GPUs.

Prints ONE JSON line on rank 0 (metric/value/unit/..., roofline, cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Gibbs sweeps/sec (full SNP pass) at N×P; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HYP = dict(sigma0=0.01, v0E=1e-4, s02E=1e-3, v0G=1e-4, s02G=1e-3)  # vignettes/BayesRR.Rmd:93-98
CVA = [1e-4, 1e-3, 1e-2]

CONFIGS = {
    "c1": dict(model="v2", N=2_000, P=10_000, groups=1,
               workload="BayesRSamplerV2 N=2,000 x P=10,000, 3-component mixture (BASELINE configs[0])"),
    "c2": dict(model="v2", N=100_000, P=500_000, groups=1,
               workload="BayesRSamplerV2 N=100,000 x P=500,000 dense f32 genotypes, 1 MI355X (BASELINE configs[1])"),
    "c3": dict(model="groups", N=100_000, P=500_000, groups=22,
               workload="BayesRSamplerV2Groups N=100,000 x P=500,000, 22 SNP groups (BASELINE configs[2])"),
    "c4": dict(model="hs", N=100_000, P=500_000, groups=1,
               workload="HorseshoeR N=100,000 x P=500,000 (BASELINE configs[3])"),
    "c5": dict(model="v2", N=500_000, P=1_000_000, groups=1,
               workload="BayesRSamplerV2 N=500,000 x P=1,000,000 column-sharded (BASELINE configs[4])"),
}


def block_events(raw, lag=1):
    """Medians over the blocks of one traced sweep.  'lat_*' are measured from the solver's
    publication of block s-1-lag's changes, which is what streaming block s waits for."""
    import numpy as np
    raw = np.asarray(raw, dtype=np.float64)
    nbk = (raw.size - 9216) // 16
    tr = raw[:nbk * 16].reshape(-1, 16)
    probe = raw[nbk * 16:nbk * 16 + 2048].reshape(2, 1024)
    acc = raw[nbk * 16 + 2048:].reshape(7, 1024)  # per streaming workgroup: wait, apply, stream; apply: list, products, part barrier, staging stores
    u64 = float(2 ** 64)
    first = lambda c: u64 - 1 - tr[:, c]  # noqa: E731  (stored as ~t)
    nb = tr.shape[0]
    if nb < 6:
        return {}
    sl = slice(4, nb - 1)
    pub_m2 = np.roll(tr[:, 3], lag + 1)
    ev = {
        "period": np.diff(tr[:, 0])[sl],
        "solver_wait": (tr[:, 1] - tr[:, 0])[sl],
        "solver_chain": (tr[:, 2] - tr[:, 1])[sl],
        "solver_publish": (tr[:, 3] - tr[:, 2])[sl],
        "lat_pend_seen_first": (first(4) - pub_m2)[sl],
        "lat_pend_seen_last": (tr[:, 5] - pub_m2)[sl],
        "lat_apply_last": (tr[:, 6] - pub_m2)[sl],
        "lat_items_first": (first(10) - pub_m2)[sl],
        "lat_items_last": (tr[:, 7] - pub_m2)[sl],
        "lat_l2_first": (first(9) - pub_m2)[sl],
        "lat_l2_last": (tr[:, 8] - pub_m2)[sl],
        "lat_solver_sees": (tr[:, 1] - pub_m2)[sl],
    }
    out = {k: round(float(np.median(v)) / 100.0, 2) for k, v in ev.items()}
    # per-workgroup probe of block nb/2: pend seen and items done, by XCD (blockIdx % 8)
    done, seen = probe[0], probe[1]
    g = np.nonzero(done)[0]
    if len(g):
        t0 = done[g].min()
        xcd = (g + 1) % 8
        out["probe_done_by_xcd"] = [round(float(np.mean(done[g][xcd == x] - t0)) / 100.0, 2) for x in range(8)]
        out["probe_seen_by_xcd"] = [round(float(np.mean(seen[g][xcd == x] - t0)) / 100.0, 2) for x in range(8)]
        out["probe_done_pct"] = [round(float(np.percentile(done[g] - t0, q)) / 100.0, 2) for q in (0, 10, 50, 90, 100)]
        out["probe_busy_pct"] = [round(float(np.percentile(done[g] - seen[g], q)) / 100.0, 2) for q in (0, 10, 50, 90, 100)]
        out["probe_slowest_wg"] = [int(x) for x in g[np.argsort(done[g] - seen[g])[-8:]]]
    # whole-sweep totals per streaming workgroup (ms): systematic vs random imbalance
    busy = acc[1] + acc[2]
    w = np.nonzero(busy)[0]
    if len(w):
        ms = lambda v: [round(float(x) / 1e5, 3) for x in v]  # noqa: E731  (100 MHz ticks)
        out["wg_wait_ms_pct"] = ms(np.percentile(acc[0][w], [0, 10, 50, 90, 100]))
        out["wg_apply_ms_pct"] = ms(np.percentile(acc[1][w], [0, 10, 50, 90, 100]))
        out["wg_stream_ms_pct"] = ms(np.percentile(acc[2][w], [0, 10, 50, 90, 100]))
        out["wg_apply_list_ms_pct"] = ms(np.percentile(acc[3][w], [0, 10, 50, 90, 100]))
        out["wg_apply_products_ms_pct"] = ms(np.percentile(acc[4][w], [0, 10, 50, 90, 100]))
        out["wg_apply_partbar_ms_pct"] = ms(np.percentile(acc[5][w], [0, 10, 50, 90, 100]))
        out["wg_apply_stage_ms_pct"] = ms(np.percentile(acc[6][w], [0, 10, 50, 90, 100]))
        out["wg_busy_by_xcd_ms"] = ms([np.mean(busy[w][(w + 1) % 8 == x]) for x in range(8)])
        out["wg_slowest"] = [int(x) for x in w[np.argsort(busy[w])[-8:]]]
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one process each).  Without WORLD_SIZE in the environment, N > 1 spawns the N "
                         "rank processes itself; with WORLD_SIZE set (torch.distributed.run) it must equal N")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed sweeps (burn-in: the first sweeps from beta = 0 change ~25%% of markers)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--P", type=int, default=None)
    ap.add_argument("--block-size", type=int, default=0,
                    help="marker block B; 0 = the library's automatic choice (512 V2, 128 Groups and Horseshoe)")
    ap.add_argument("--order", default="blocked", choices=["blocked", "reference"],
                    help="visit order: BLOCKED (fast path) or the reference's own std::random_shuffle order "
                         "(Gram blocks recomputed every sweep)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--data-seed", type=int, default=20261015)
    ap.add_argument("--profile-solve", action="store_true", help="k_solve phase timers (diag)")
    ap.add_argument("--trace-sweeps", type=int, default=0, help="time N more sweeps one by one (diag)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-markers", type=int, default=3000,
                    help="markers in the bounded CPU-baseline sample (N as in the config)")
    ap.add_argument("--cpu-sweeps", type=int, default=2, help="sweeps per timed repeat of the CPU sample")
    ap.add_argument("--cpu-repeats", type=int, default=3, help="timed repeats of the CPU sample (median reported)")
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-roofline-events", action="store_true")
    ap.add_argument("--exchanges", type=int, default=0,
                    help="column shards: residual exchanges per sweep E (0 = the library's automatic E = 8, whose "
                         "8-shard chain matches the 1-shard chain; 1 = north_star's one all-reduce per sweep, "
                         "biased from 2 shards on; DESIGN.md section 9)")
    ap.add_argument("--rank-of", type=int, default=0, metavar="S",
                    help="measurement: time ONE rank's real workload of an S-GPU column-sharded job on this GPU "
                         "(shard 0 of S, every exchange segment, BRR_EXCHANGE_LOOPBACK=1: the other ranks' deltas "
                         "taken as zero, so no collective); not a whole-job number")
    ap.add_argument("--shard", default="cols", choices=["cols", "rows"],
                    help="N > 1: column shards with one residual all-reduce per sweep (north_star, SURVEY 8e; "
                         "default) or exact row shards with an all-reduce of each block's dots (SURVEY 8f4)")
    ap.add_argument("--emit", default=None, metavar="PATH",
                    help="output-on run (BASELINE.md): write the reference CSV of every --emit-thin'th timed sweep "
                         "through the asynchronous sample pipeline (SURVEY 8f2), drained inside the timed region")
    ap.add_argument("--emit-thin", type=int, default=10, help="thinning of the output-on run (vignette: 10)")
    ap.add_argument("--oneshot", action="store_true",
                    help="C1 as BASELINE.md states it: the drop-in one-shot brr_BayesRSamplerV2 on host data "
                         "(N=2,000 x P=10,000, 1,000 iterations, burn-in 500, thinning 10, CSV written), timed "
                         "end to end, beside the CPU oracle's one-shot on the same data")
    ap.add_argument("--cpu-iters", type=int, default=100,
                    help="--oneshot: iterations of the CPU oracle's run (extrapolated to the full run; "
                         "0 = the full max_iterations)")
    ap.add_argument("--x-storage", default="f32", choices=["f32", "2bit"],
                    help="genotype storage on the device: dense f32 (the BASELINE configs) or 2-bit codes "
                         "+ per-column value tables (SURVEY 8f3; decoded values identical to f32)")
    return ap.parse_args()


# ------------------------------------------------------------------------------------------
def cpu_baseline_child(args):
    """Runs in a subprocess pinned to ONE core: the reference-faithful CPU oracle (f64, y~
    materialised, single thread -- the reference's package build is single-threaded,
    SURVEY fact 5) on a bounded sample of the same workload."""
    core = sorted(os.sched_getaffinity(0))[0]
    os.sched_setaffinity(0, {core})
    from oracle import oracle as O
    O.build()
    cfg = CONFIGS[args.config]
    N = args.N or cfg["N"]
    Pm = args.cpu_markers
    X = O.synth_x(args.data_seed, N, Pm)
    import numpy as np
    rng = np.random.default_rng(0)
    Y = rng.normal(size=N)
    Y = (Y - Y.mean()) / Y.std(ddof=1)
    kw = dict(HYP)
    model = {"v2": O.V2, "groups": O.GROUPS, "hs": O.HORSESHOE}[cfg["model"]]
    if cfg["model"] == "hs":
        kw = dict(A=(1 / N ** 0.5) * 1500 / (cfg["P"] - 1500), v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0,
                  c2=1.0, vC=10.0, sC=10.0)
    elif cfg["model"] == "groups":
        import numpy as np
        G = cfg["groups"]
        kw.update(G=G, cva=np.tile(CVA, (G, 1)), gAssign=(np.arange(Pm) * G // Pm).astype(np.int32),
                  fixed=np.zeros((N, 1)))
    else:
        kw.update(cva=CVA)
    o = O.Oracle(model, X, Y, seed=args.seed, order_mode=O.ORDER_REFERENCE, **kw)
    o.sweep(1)  # warm
    load0 = _loadavg()
    runs = []
    for _ in range(max(1, args.cpu_repeats)):  # repeats: the host's load moves a single run by up to 2x
        t0 = time.perf_counter()
        o.sweep(args.cpu_sweeps)
        runs.append((time.perf_counter() - t0) / args.cpu_sweeps)
    print(json.dumps({"t_sweep_runs_s": runs, "markers": Pm, "N": N, "core": core,
                      "loadavg_before": load0, "loadavg_after": _loadavg()}))


def _loadavg():
    try:
        with open("/proc/loadavg") as f:
            return " ".join(f.read().split()[:3])
    except OSError:
        return None


def pmc_traffic(args, N, P, B, fused, x_bytes):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary of the
    same configuration (profiles/*_pmc.json, written by scripts/pmc_json.py: FETCH_SIZE x2 +
    WRITE_SIZE, gfx950 correction), or None."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")), reverse=True):  # newest round first
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (d.get("config") == args.config and d.get("block_size") == B and fused
                and d.get("x_storage", "f32") == args.x_storage
                and d.get("algorithmic_bytes_per_launch") == x_bytes):
            return d["hbm_bytes_per_launch"], os.path.relpath(f, REPO)
    return None, None


def host_cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args, P_full):
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--config", args.config,
           "--cpu-markers", str(args.cpu_markers), "--cpu-sweeps", str(args.cpu_sweeps),
           "--cpu-repeats", str(args.cpu_repeats),
           "--data-seed", str(args.data_seed)]
    if args.N:
        cmd += ["--N", str(args.N)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        return {"value": None, "unit": "sweeps/s", "cores": 1, "kind": "port",
                "sample": f"failed: {out.stderr[-300:]}"}
    r = json.loads(out.stdout.strip().splitlines()[-1])
    tm = sorted(t / r["markers"] for t in r["t_sweep_runs_s"])
    t_marker = tm[len(tm) // 2]  # median of the repeats
    return {
        "value": 1.0 / (t_marker * P_full),
        "unit": "sweeps/s (extrapolated: 1 / (P x median t_marker))",
        "cores": 1,
        "kind": "port",
        "host_cpu": host_cpu_model(), "host_nproc": os.cpu_count(),
        "sample": (f"CPU oracle (reference-faithful C restatement, f64, y~ materialised, 1 thread "
                   f"pinned to core {r['core']}) N={r['N']} x {r['markers']} markers, {len(tm)} repeats of "
                   f"{args.cpu_sweeps} sweeps; median t_marker={t_marker * 1e3:.4f} ms; P={P_full}"),
        "t_marker_ms": t_marker * 1e3,
        "t_marker_min_ms": tm[0] * 1e3,
        "t_marker_runs_ms": [round(t * 1e3, 4) for t in tm],
        "value_at_min": 1.0 / (tm[0] * P_full),
        "pinned_core": r["core"],
        "host_loadavg": [r["loadavg_before"], r["loadavg_after"]],
    }


# ------------------------------------------------------------------------------------------
def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """--gpus N without a launcher: start N fresh rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1) and exit with the worst
    return code.  This parent never touches the GPU, so nothing is exec'd from a GPU process."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def c1_data(N, P, seed):
    """Host synthetic cohort of the BASELINE spec (numpy: Binomial(2, f), f ~ U(0.05, 0.5), columns
    standardised with the N-1 sd, min(1000, P/10) causal effects, h2 = 0.5, Y standardised)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    f = rng.uniform(0.05, 0.5, P)
    G = rng.binomial(2, f, size=(N, P)).astype(np.float64)
    sd = G.std(axis=0, ddof=1)
    G = (G - G.mean(axis=0)) / np.where(sd > 0, sd, 1.0)
    X = np.asfortranarray(G.astype(np.float32).astype(np.float64))
    nc = max(1, min(1000, P // 10))
    b = np.zeros(P)
    b[rng.choice(P, nc, replace=False)] = rng.normal(0, np.sqrt(0.5 / nc), nc)
    y = X @ b + rng.normal(0, np.sqrt(0.5), N)
    return X, (y - y.mean()) / y.std(ddof=1)


def cpu_oneshot_child(args):
    """--oneshot CPU leg (one pinned core): the oracle's reference-faithful one-shot."""
    import numpy as np
    os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    from oracle import oracle as O
    O.build()
    X, Y = c1_data(2000, 10000, args.data_seed)
    it = args.cpu_iters
    t0 = time.perf_counter()
    O.run_csv("/tmp/brr_c1_cpu.csv", O.V2, X, Y, it, it // 2, 10, cva=CVA, seed=args.seed, order_mode=0, **HYP)
    print(json.dumps({"t_s": time.perf_counter() - t0, "iters": it}))


def main_oneshot(args):
    """C1 (BASELINE configs[0]) through the drop-in entry point, end to end."""
    import numpy as np
    import bayesrrcpp_amd as B
    N, P, MAXIT, BURN, THIN = 2000, 10000, 1000, 500, 10
    X, Y = c1_data(N, P, args.data_seed)
    out = os.path.join(REPO, "gpurun_out", "c1_oneshot.csv")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    B.BayesRSamplerV2(out, args.seed, 5, 1, 1, X[:, :512].copy(order="F"), Y, HYP["sigma0"], HYP["v0E"],
                      HYP["s02E"], HYP["v0G"], HYP["s02G"], CVA, log=lambda m: None)  # warm (module load)
    # host-side timeline of the timed call (libbrr BRR_TIMELINE: one line per phase and per 100
    # iterations, through the log callback)
    os.environ["BRR_TIMELINE"] = "1"
    tl = []
    t0 = time.perf_counter()
    B.BayesRSamplerV2(out, args.seed, MAXIT, BURN, THIN, X, Y, HYP["sigma0"], HYP["v0E"], HYP["s02E"],
                      HYP["v0G"], HYP["s02G"], CVA, log=lambda m: tl.append(m.rstrip()) if m.startswith("timeline") else None)
    dt = time.perf_counter() - t0
    os.environ.pop("BRR_TIMELINE")
    rows = sum(1 for _ in open(out)) - 1
    cpu = None
    if not args.no_cpu_baseline:
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--oneshot",
               "--cpu-iters", str(args.cpu_iters or MAXIT), "--data-seed", str(args.data_seed), "--seed", str(args.seed)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=3000)
        if r.returncode == 0:
            c = json.loads(r.stdout.strip().splitlines()[-1])
            cpu = {"value": c["iters"] / c["t_s"], "unit": "sweeps/s" + (" (extrapolated from a shorter run)"
                                                                          if c["iters"] < MAXIT else ""),
                   "cores": 1, "kind": "port", "host_cpu": host_cpu_model(), "host_nproc": os.cpu_count(),
                   "sample": f"CPU oracle one-shot (reference-faithful C restatement, 1 pinned core), "
                             f"{c['iters']} iterations of the same data, CSV written, {c['t_s']:.1f} s"}
        else:
            cpu = {"value": None, "sample": "failed: " + r.stderr[-300:]}
    print(json.dumps({
        "metric": METRIC, "value": round(MAXIT / dt, 3), "unit": "sweeps/s (end to end: upload, init, 1,000 sweeps, CSV)",
        "n_gpus": 1, "steps": MAXIT, "warmup": 0, "ms_per_step": round(dt / MAXIT * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic host cohort (numpy Binomial(2,f), standardised, f32-representable), f64 arithmetic",
        "config": {"workload": "C1: brr_BayesRSamplerV2 one-shot N=2,000 x P=10,000, 1,000 iterations, burn-in 500, "
                               "thinning 10 (BASELINE configs[0], vignettes/BayesRR.Rmd:93-100)",
                   "wall_s": round(dt, 3), "csv_rows": rows, "csv_bytes": os.path.getsize(out), "timeline": tl},
        "roofline": None, "cpu_baseline": cpu}), flush=True)


def main():
    args = parse()
    if args.cpu_baseline_child and args.oneshot:
        cpu_oneshot_child(args)
        return
    if args.cpu_baseline_child:
        cpu_baseline_child(args)
        return
    if args.oneshot:
        main_oneshot(args)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            sys.exit(spawn_ranks(args.gpus))
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to time a mislabelled run")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config == "c5" and world == 1 and args.rank_of <= 1:
        # C5's 2 TB of f32 genotypes need 8 GPUs: on one GPU, time one rank's real share of it
        print("bench.py: --config c5 on one GPU times rank 0 of 8 (--rank-of 8)", file=sys.stderr)
        args.rank_of = 8
    emu = args.rank_of if world == 1 and args.rank_of > 1 else 0  # one rank of an emu-GPU job, emulated
    if emu:
        os.environ["BRR_EXCHANGE_LOOPBACK"] = "1"
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo only: rendezvous / barrier / max-over-ranks
        dist.init_process_group("gloo")
    import numpy as np
    import bayesrrcpp_amd as B
    from bayesrrcpp_amd import _lib as L
    from bayesrrcpp_amd.session import comm_unique_id

    cfg = CONFIGS[args.config]
    N = args.N or cfg["N"]
    P = args.P or cfg["P"]
    model = {"v2": L.MODEL_V2, "groups": L.MODEL_GROUPS, "hs": L.MODEL_HORSESHOE}[cfg["model"]]
    Bsz = args.block_size or (128 if model in (L.MODEL_HORSESHOE, L.MODEL_GROUPS) or N < 32768 or args.order == "reference"
                              else 512)  # = libbrr's automatic B
    G = cfg["groups"]
    K = 1 if model == L.MODEL_HORSESHOE else len(CVA) + 1
    F = 1 if model == L.MODEL_GROUPS else 0
    x2 = args.x_storage == "2bit"
    order_mode = L.ORDER_REFERENCE if args.order == "reference" else L.ORDER_BLOCKED
    rows = args.shard == "rows" and world > 1
    if rows:
        # exact row shards: rows [r0, r1) of the cohort, every marker
        r0, r1 = N * rank // world, N * (rank + 1) // world
        c0, c1, Pl, Nl = 0, P, P, r1 - r0
        s = B.Session(model, Nl, P, K=K, groups=G, F=F, device=local_rank, block_size=Bsz,
                      order_mode=order_mode, row_shard_rank=rank, row_shard_count=world, row_offset=r0,
                      N_total=N, x_storage=L.X_2BIT if x2 else L.X_F32)
    else:
        # contiguous block shards (--rank-of S: shard 0 of S on this one GPU)
        nshard, srank = (emu, 0) if emu else (world, rank)
        nb = (P + Bsz - 1) // Bsz
        b0, b1 = nb * srank // nshard, nb * (srank + 1) // nshard
        c0, c1 = b0 * Bsz, min(P, b1 * Bsz)
        Pl, Nl = c1 - c0, N
        s = B.Session(model, N, Pl, K=K, groups=G, F=F, M_total=P, col_offset=c0, device=local_rank,
                      block_size=Bsz, order_mode=order_mode, shard_rank=srank, shard_count=nshard,
                      x_storage=L.X_2BIT if x2 else L.X_F32, exchanges_per_sweep=args.exchanges)
    n_ex = s.exchanges_per_sweep

    def diag_scalar(k, default=0):
        """a diagnostic scalar of the library (not in brr.h); an older library build lacks some"""
        try:
            return s.scalar(k)
        except Exception:  # noqa: BLE001 -- older libbrr (A/B runs): the field is absent
            return default
    # algorithmic bytes of one pass over this shard's genotypes (f32 values, or 2-bit codes + the
    # 16-B value table of every column)
    x_bytes = (Nl * Pl / 4.0 + 16.0 * Pl) if x2 else 4.0 * Nl * Pl
    t_setup = time.perf_counter()
    s.synthesize(args.data_seed, 0.5, -1)
    if world > 1 and rows:
        parts = [None] * world
        dist.all_gather_object(parts, s.synth_partial_y())
        s.synth_y(np.concatenate(parts), args.data_seed, 0.5)
    elif world > 1:
        import torch
        g = torch.from_numpy(s.synth_partial_y())
        dist.all_reduce(g)
        s.synth_y(g.numpy(), args.data_seed, 0.5)
    elif emu:  # Y from this shard's genetic values (the other shards' parts taken as zero)
        s.synth_y(s.synth_partial_y(), args.data_seed, 0.5)
    if model == L.MODEL_HORSESHOE:
        s.set_horseshoe(A=(1 / N ** 0.5) * 1500 / (P - 1500), v0E=1e-3, s02E=1e-3, vL=1.0, vT=1.0,
                        c2=1.0, vC=10.0, sC=10.0)  # HorseshoeR.cpp:315-323
    else:
        gA = (np.arange(c0, c1) * G // P).astype(np.int32) if G > 1 else None
        s.set_bayesr(cva=np.tile(CVA, (G, 1)), gAssign=gA, **HYP)
        if F:
            s.set_fixed(np.zeros((N, F)))  # vignettes/BayesRR.Rmd:166: one all-zero column
    if world > 1:  # (row shards sum their Gram blocks inside init: the communicator comes first)
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        s.comm_init(uid[0], world, rank)
    s.init(args.seed)
    s.synchronize()
    t_setup = time.perf_counter() - t_setup

    def barrier():
        s.synchronize()
        if dist is not None:
            dist.barrier()

    warm_trace = []
    if args.trace_sweeps:
        c0 = s.scalar(101)
        for _ in range(args.warmup):
            t1 = time.perf_counter()
            s.sweep(1)
            s.synchronize()
            c1 = s.scalar(101)
            warm_trace.append((round((time.perf_counter() - t1) * 1e3, 2), int(c1 - c0)))
            c0 = c1
    else:
        s.sweep(args.warmup)
    barrier()
    emit = None
    t0 = time.perf_counter()
    if args.emit:
        path = args.emit if world == 1 else f"{args.emit}.rank{rank}"
        s.output_open(path, header=True, ring_depth=4)
        rows = 0
        for k in range(args.steps):
            s.sweep(1)
            if k % args.emit_thin == 0:
                s.output_sample(args.warmup + k)
                rows += 1
        inflight = s.output_close()  # every row formatted and written
        emit = {"path": path, "thinning": args.emit_thin, "rows": rows, "max_rows_in_flight": inflight,
                "bytes": os.path.getsize(path)}
    else:
        s.sweep(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms = dt / args.steps * 1e3
    # fingerprint of the chain's state after the timed sweeps (A/B runs of library variants that must give
    # the same chain compare it)
    import hashlib
    state_sha = hashlib.sha256(s.vector(L.BETA).tobytes() + s.vector(L.EPS).tobytes()).hexdigest()[:16]
    if diag_scalar(130) > 0:  # the fused sweep fell back to the per-block kernels: say so, loudly
        print(f"bench.py: WARNING: {int(diag_scalar(130))} fused sweep(s) failed the residency census; the "
              "session ran the per-block kernels afterwards (see config.census_failures)", file=sys.stderr)
    diag = {"state_sha16": state_sha, "slow_steps_per_sweep": s.scalar(100) / (args.warmup + args.steps),
            "changed_per_sweep": s.scalar(101) / (args.warmup + args.steps),
            "nonzero_frac": 1.0 - float(s.vector(L.VCOUNT)[0]) / P if model != L.MODEL_HORSESHOE else 1.0}
    value = args.steps / dt  # whole-job sweeps/s (every rank holds a shard of the same sweep)

    # roofline of the dominant kernel (k_stream): HIP events around every streaming launch on
    # the session stream, over a few instrumented sweeps after the timed region
    roof = None
    if not args.no_roofline_events:
        # roofline of the dominant kernel, timed with HIP events on the session stream over two
        # instrumented sweeps after the timed region.  Fused mode: k_sweep is ONE launch per
        # sweep that streams this shard's whole X once (algorithmic bytes 4 N P); per-block mode:
        # k_stream streams one block (4 N B) per launch.
        fused = s.scalar(104) > 0
        s.set_timing(True)
        s.sweep(2)
        tm = s.timing()
        s.set_timing(False)
        nbl = (Pl + Bsz - 1) // Bsz
        if fused or rows:
            launches = max(1, tm["stream_launches"] // nbl)
            bytes_launch = x_bytes
            kname = ("row-shard marker loop (per block: k_stream, k_slab_total, ncclAllReduce of the B dots, k_solve)"
                     if rows else "k_sweep_solve + k_sweep_stream (fused marker loop: solver, streaming and reducing workgroups)")
        else:
            launches = max(1, tm["stream_launches"])
            bytes_launch = x_bytes * Bsz / Pl
            kname = "k_stream"
        avg_ms = tm["stream_ms"] / launches
        achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(args, N, Pl, Bsz, fused, x_bytes)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "kernel": kname, "avg_launch_us": round(avg_ms * 1e3, 3),
                "bytes_per_launch": int(bytes_launch),
                "per_block_us": round(tm["stream_ms"] / max(1, tm["stream_launches"]) * 1e3, 3),
                "sweep_hbm_gbs": round(x_bytes / (ms * 1e-3) / 1e9, 1),
                # what limits this configuration in measurement; frac is
                # always against the HBM roofline of the algorithmic bytes
                "limiter": ("solver workgroup per 512-marker block (decisions incl. the dots poll, Gram-row staging, row chain, write-back); the decode-dot is not the bound" if x2 and model not in (L.MODEL_GROUPS, L.MODEL_HORSESHOE)
                            else "solver workgroup's serial chain (overlapped solver: the next block's decisions, Gram block and corrections prepared beside it)" if model == L.MODEL_GROUPS
                            else "streaming workgroups: the dense apply of every column from the LDS class-code cache plus the stream; the solver close behind" if model == L.MODEL_HORSESHOE
                            else "HBM stream")}
    if args.trace_sweeps:
        # per-sweep wall time and changed markers of a fresh chain's first sweeps (diagnostic)
        tr = []
        s2 = s
        c0 = s2.scalar(101)
        for _ in range(args.trace_sweeps):
            t1 = time.perf_counter()
            s2.sweep(1)
            s2.synchronize()
            c1 = s2.scalar(101)
            tr.append((round((time.perf_counter() - t1) * 1e3, 2), int(c1 - c0)))
            c0 = c1
        diag["sweep_trace_ms_changed"] = {"warmup": warm_trace, "after": tr}
    if args.profile_solve:
        # k_solve phase breakdown (device wall clock, 100 MHz) over two more sweeps
        s.set_scalar(102, 1.0)
        s.sweep(2)
        calls = max(1.0, s.scalar(115))
        diag["solve_phase_us"] = {k: round(s.scalar(110 + i) / calls / 100.0, 3) for i, k in
                                  enumerate(["load", "gram_rows", "chain", "writeback"])}
        diag["solve_chain_steps"] = round(s.scalar(116) / calls, 2)
        diag["solve_refreshes"] = round(s.scalar(117) / calls, 2)
        diag["solve_global_rows"] = round(s.scalar(114) / calls, 2)
        diag["solve_refresh_us"] = round(s.scalar(118) / calls / 100.0, 3)
        diag["solve_correct_us"] = round(s.scalar(119) / calls / 100.0, 3)
        diag["solve_wait_us"] = round(s.scalar(120) / calls / 100.0, 3)
        # phase A (thread 0's view): constants, cross-Gram correction, resident coefficients
        diag["solve_phaseA_us"] = {k: round(s.scalar(123 + i) / calls / 100.0, 3) for i, k in
                                   enumerate(["constants", "correction", "coefficients"])}
        # shader clock during the chain: s_memtime ticks / s_memrealtime (100 MHz) ticks
        diag["solve_chain_clock_ghz"] = round(s.scalar(121) / max(1.0, s.scalar(112)) * 0.1, 3)
        # serial chain loop alone (shader clocks per chain step; wave 0 of the solver)
        diag["solve_chain_loop_cycles_per_step"] = round(s.scalar(122) / max(1.0, s.scalar(116)), 1)
        # (B >= 256 row chain) chain end -> every wave past the barrier, ring rows, predicted positions
        diag["solve_after_chain_us"] = round(s.scalar(127) / calls / 100.0, 3)
        diag["solve_ring_rows"] = round(s.scalar(128) / calls, 2)
        diag["solve_predicted"] = round(s.scalar(129) / calls, 2)
        # streamer boundaries whose change list was prefetched (per streaming workgroup and block)
        nsg_ = int(s.scalar(104))
        if nsg_ > 0:
            diag["list_prefetch_frac"] = round(s.scalar(126) / (2.0 * nsg_ * max(1, -(-P // Bsz))), 3)
        if int(s.scalar(104)) > 0:
            # per-block event trace of one fused sweep (brr_kernels.hip TR_*), medians in us
            s.set_scalar(102, 1.0)
            s.sweep(1)
            diag["block_events_us"] = block_events(s.vector(201), int(s.scalar(106)))
        s.set_scalar(102, 0.0)
    cpu = None
    if rank == 0 and world == 1 and not emu and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, P)
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 4), "unit": "sweeps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": ("synthetic (on-device Binomial(2,f) genotypes, standardised; "
                     + ("2-bit codes + f32 value tables" if x2 else "f32 X") + ", f64 arithmetic)"),
            "config": {"workload": cfg["workload"] + (" [2-bit genotype storage, SURVEY 8f3]" if x2 else ""),
                       "x_storage": args.x_storage, "N": N, "P": P, "K": K, "groups": G,
                       "block_size": Bsz, "order": args.order, "fused_stream_wg": int(s.scalar(104)), "code_cache": int(s.scalar(105)), "pipeline_lag": int(s.scalar(106)), "stream_wg_threads": int(diag_scalar(109)), "reducer_wg": int(diag_scalar(131)),
                       "census_failures": int(diag_scalar(130)),
                       "parallelism": (f"row-shard x{world} (exact)" if rows
                                       else f"column-shard rank 0 of {emu} emulated on 1 GPU, {n_ex} exchanges per sweep "
                                            f"(other ranks' deltas zero, no collective; a per-rank rate, not a whole-job one)"
                                       if emu else f"column-shard x{world}" + (f", {n_ex} exchanges per sweep" if world > 1 else "")),
                       "setup_s": round(t_setup, 2), "diag": diag,
                       **({"output": emit} if emit else {})},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    s.synchronize()
    s.close()  # device resources released while the runtime (and a profiler's tool) is still up
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
