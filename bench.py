"""Benchmark: Option.carry_out transitions/s, batched 6-player self-play.

Workload (BASELINE.json configs[1], "config 2"): per GPU, 4096 preset
6-player games (run_utils.create_game) played by the uniform random policy
to terminal.  One bench step = one launch of the fused rollout kernel
(k_rollout_u) over a fresh batch of 4096 games already resident in HBM
(initialised, untimed, before the timed region); seeds are disjoint across
steps and ranks (seed = base + (step * world + rank) * B + lane), so N GPUs
play N x 4096 independent games per step (weak scaling, no data-path
collective).  The K steps are launched round-robin on `--streams` HIP
streams (default 3, warmed before the timed region): a launch lasts as long
as its longest game, and the next batch's games take the SIMD slots the
finished games free (tests/test_gpu_parity.py::test_gpu_rollout_streams_overlap
checks overlapped batches equal batches run alone).  `streams.one_stream`
replays the same K batches one after another for comparison.

Prints ONE JSON line on rank 0.  `value` = carry_out transitions of all ranks
/ max-over-ranks wall time of the K timed steps.

* `roofline` prices one k_rollout_u launch running alone (the one-stream
  replay; the PMC children run with --streams 1) by its algorithmic bytes (2 x CIT_GAME_BYTES
  per transition) over its HIP-event duration against HBM
  peak; `traffic` is the HBM bytes per launch measured IN THIS RUN by two
  rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short child run of
  this script (N = 1 only; gfx950 FETCH_SIZE half-count corrected).  Since
  the kernel keeps each game in LDS, those bytes are far below the
  algorithmic ones: `roofline.issue` reports what does bound it, from a third
  --pmc pass of SQ counters: SALU / VALU / LDS instructions per transition,
  the scalar-issue floor (1 SALU per clock per CU) and the wait fraction.
* `cpu_baseline` times the build's C++ CPU restatement (the same engine
  headers compiled with g++, build/libcitadels_hostcheck.so) on 1 host core
  and on all the cores this process may use, on rank 0 at N = 1, with nproc
  and the lscpu model; the pure-Python oracle (oracle/) is a secondary
  figure and the reference's own Python is quoted from BASELINE.md (measured
  in the survey container; it cannot travel to the GPU box).
* `e2e` adds the untimed init: games/s with k_init (seeding + deal) inside
  the timed region.
* `roofline.latency`: one wave runs one game, so a launch lasts as long as
  its longest game; steps_mean / steps_max is the share of the launch a
  SIMD slot does useful work, and kernel time / steps_max the per-step
  latency of that game (tools/rollout_clock.py).
"""
import argparse
import ctypes as C
import glob
import csv
import json
import multiprocessing as mp
import os
import platform
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
N_CU, CLOCK_HZ, SIMD_PER_CU = 256, 2.4e9, 4
BASE_SEED = 1_000_000_000
KERNEL = "k_rollout_u"
# The reference's own Python, BASELINE.md §2 config 1 (survey container, 8-core Xeon).
REF_PY = {"1_core": 12301, "8_procs": 83869, "unit": "carry_out transitions/s",
          "where": "survey container (BASELINE.md), not this box"}
SQ_SET = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
          "SQ_BUSY_CYCLES", "SQ_INSTS_SMEM"]


def _oracle_worker(args):
    seed0, budget_s = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import citadels_oracle as O
    t0 = time.perf_counter()
    steps = games = 0
    s = seed0
    while time.perf_counter() - t0 < budget_s:
        try:
            _, n = O.random_rollout(s, True)
        except Exception:
            n = 0
        steps += n
        games += 1
        s += 1
    return steps, games, time.perf_counter() - t0


def host_threads():
    """Cores this process may use: the affinity set, capped by OMP_NUM_THREADS
    (the GPU box's CPU share is 16 of a much larger machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(seconds, py_seconds):
    """the build's C++ CPU restatement on 1 core and on all usable
    cores, plus the Python oracle (secondary)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import hostcheck
    lib = hostcheck.lib()
    lib.cith_rollout_timed.argtypes = [C.c_int, C.c_uint64, C.c_double, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.cith_rollout_timed.restype = C.c_int
    threads = host_threads()
    legs = {}
    for name, th in (("1_core", 1), ("all_cores", threads)):
        g, st, w = C.c_longlong(), C.c_longlong(), C.c_double()
        err = lib.cith_rollout_timed(1, C.c_uint64(BASE_SEED + 10**9), C.c_double(seconds), th, C.byref(g),
                                     C.byref(st), C.byref(w))
        legs[name] = {"value": st.value / w.value, "threads": th, "games": g.value, "transitions": st.value,
                      "wall_s": w.value, "lane_errors": err}
    ctx = mp.get_context("spawn")
    procs = threads
    with ctx.Pool(procs) as pool:
        res = pool.map(_oracle_worker, [(BASE_SEED + 10**8 + i * 10**6, py_seconds) for i in range(procs)])
    py = {"value": sum(r[0] for r in res) / max(r[2] for r in res), "procs": procs,
          "games": sum(r[1] for r in res), "kind": "port (pure-Python oracle/citadels_oracle.py)"}
    a = legs["all_cores"]
    return {"value": a["value"], "unit": "carry_out transitions/s", "cores": a["threads"], "kind": "port",
            "impl": "cpp-restatement: the engine headers (csrc/cit_engine.h) built with g++ -O3 for the host, "
                    "one game per thread",
            "sample": "%d preset games, uniform random policy to terminal, %d threads x %.0f s (all cores) and "
                      "%d games on 1 core x %.0f s" % (a["games"], a["threads"], seconds, legs["1_core"]["games"],
                                                     seconds),
            "one_core": legs["1_core"]["value"], "legs": legs, "nproc": os.cpu_count(),
            "usable_cores": threads, "cpu_model": cpu_model(), "python_oracle": py,
            "reference_python": REF_PY}


def _rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def _pmc_pass(counters, outdir, timeout_s=150):
    """One rocprofv3 --pmc pass over a short child run of this script (its own
    process group, killed on timeout).  Returns {counter: mean per launch of
    k_rollout_u} or raises."""
    os.makedirs(outdir, exist_ok=True)
    cmd = ["rocprofv3", "--pmc"] + counters + ["--output-format", "csv", "-d", outdir, "-o", "run", "--",
                                              sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2",
                                              "--warmup", "1", "--streams", "1", "--no-cpu-baseline",
                                              "--no-pmc"]
    env = dict(os.environ, TMPDIR="/tmp")
    with open(os.path.join(outdir, "log.txt"), "w") as log:
        p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
        try:
            rc = p.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            raise RuntimeError("rocprofv3 --pmc %s timed out" % counters)
    if rc != 0:
        raise RuntimeError("rocprofv3 --pmc %s exited %d" % (counters, rc))
    per = {}
    for r in _rows(os.path.join(outdir, "**", "*counter_collection.csv")):
        if KERNEL in r.get("Kernel_Name", ""):
            per.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id", "0"), 0.0)
            per[r["Counter_Name"]][r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
    if not per:
        raise RuntimeError("no %s rows in the rocprofv3 output" % KERNEL)
    return {k: sum(v.values()) / len(v) for k, v in per.items()}


def pmc_in_run():
    """Three --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ set), each its own child run."""
    base = tempfile.mkdtemp(prefix="bench_pmc_", dir="/tmp")
    out = {"source": "in-run rocprofv3 --pmc, 3 passes over `bench.py --steps 2 --warmup 1` children"}
    try:
        f = _pmc_pass(["FETCH_SIZE"], os.path.join(base, "fetch"))["FETCH_SIZE"]
        w = _pmc_pass(["WRITE_SIZE"], os.path.join(base, "write"))["WRITE_SIZE"]
        out["fetch_size_kib"] = f
        out["write_size_kib"] = w
        out["hbm_bytes_per_launch"] = 2 * 1024 * f + 1024 * w
        out["sq"] = _pmc_pass(SQ_SET, os.path.join(base, "sq"))
    except Exception as e:  # a missing profiler must not cost the bench line
        out["error"] = str(e)[:300]
    return out


def issue_roofline(sq, trans_per_launch, kernel_ms):
    """What bounds k_rollout_u: instruction issue, from the SQ counters (per
    wave instruction counts; SQ_*_CYCLES in quad-cycles, used only as a ratio)."""
    if not sq or "SQ_INSTS_SALU" not in sq:
        return None
    salu, valu, lds = sq["SQ_INSTS_SALU"], sq.get("SQ_INSTS_VALU", 0.0), sq.get("SQ_INSTS_LDS", 0.0)
    salu_floor_ms = salu / (N_CU * CLOCK_HZ) * 1e3                     # 1 scalar issue / clk / CU
    valu_floor_ms = valu * 4 / (N_CU * SIMD_PER_CU * CLOCK_HZ) * 1e3    # wave64 on SIMD16: 4 clk
    out = {"bound": "salu-issue", "salu_per_transition": salu / trans_per_launch,
           "valu_per_transition": valu / trans_per_launch, "lds_per_transition": lds / trans_per_launch,
           "salu_floor_ms": salu_floor_ms, "valu_floor_ms": valu_floor_ms,
           "frac": salu_floor_ms / kernel_ms,
           "model": "floor = SQ_INSTS_SALU / (256 CU x 2.4 GHz x 1 SALU/clk); frac = floor / kernel time"}
    if sq.get("SQ_WAVE_CYCLES"):
        out["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0.0) / sq["SQ_WAVE_CYCLES"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="games per GPU")
    ap.add_argument("--games-per-block", type=int, default=0, help="0 = k_rollout_u (one game per workgroup)")
    ap.add_argument("--streams", type=int, default=3,
                    help="HIP streams the K timed batches are launched round-robin on (1 = one after another)")
    ap.add_argument("--cpu-seconds", type=float, default=5.0, help="per C++ CPU-baseline leg")
    ap.add_argument("--py-seconds", type=float, default=2.0, help="Python-oracle CPU figure")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the in-run rocprofv3 --pmc passes")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the real path); gloo only to rehearse N>1 ranks on one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()          # does not initialise the GPU
    # One rank per GPU.  More ranks than GPUs is only a rehearsal: the ranks are
    # folded onto the visible GPUs and the line says so ("folded").
    folded = world > max(1, n_dev)
    if folded and args.dist_backend == "nccl":
        raise SystemExit("bench.py: WORLD_SIZE=%d > %d visible GPUs; RCCL needs one rank per GPU "
                         "(use --dist-backend gloo to rehearse folded ranks)" % (world, n_dev))

    # The PMC passes run as child processes before this process touches the GPU.
    pmc = pmc_in_run() if (world == 1 and not args.no_pmc) else None

    dev = torch.device("cuda", local % max(1, n_dev))
    if world > 1:
        torch.cuda.set_device(dev)
        dist.init_process_group(args.dist_backend)
    torch.cuda.set_device(dev)

    from citadels_self_play_amd import layout as L
    from citadels_self_play_amd.engine import GameBatch

    B, K, W, S = args.batch, args.steps, args.warmup, max(1, args.streams)
    seer = None
    batches = []
    for step in range(W + K):
        s0 = BASE_SEED + (step * world + rank) * B
        gb = GameBatch(np.arange(s0, s0 + B), preset=True, device=dev, games_per_block=args.games_per_block,
                       seer=seer)
        if S == 1:          # the seer scratch is per lane: batches in flight together need their own
            seer = gb.seer
        batches.append(gb)
    torch.cuda.synchronize()

    for gb in batches[:W]:
        gb.rollout()
    torch.cuda.synchronize()

    # HIP events on the stream each kernel is launched on.  With S > 1 streams
    # batch k goes to stream k % S, so the next batches' games take the SIMD
    # slots the finished games of earlier batches leave (the launch tail).
    stream = torch.cuda.current_stream()
    streams = [stream] if S == 1 else [torch.cuda.Stream(device=dev) for _ in range(S)]
    if S > 1:
        # A stream's first launches set up its hardware queue: warm every stream
        # with a small rollout of its own (untimed, seeds outside the timed ones).
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                for _ in range(2):
                    GameBatch(np.arange(BASE_SEED - (i + 1) * 256, BASE_SEED - i * 256), preset=True, device=dev,
                              games_per_block=args.games_per_block).rollout()
        torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, gb in enumerate(batches[W:]):
        st = streams[k % S]
        with torch.cuda.stream(st):
            evs[k][0].record(st)
            gb.rollout()
            evs[k][1].record(st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    trans_rank = sum(int(gb.steps.sum().item()) for gb in batches[W:])
    serial = None
    if S > 1:
        # The roofline prices one launch running alone: replay the same K
        # batches one after another on one stream (re-initialised, untimed init).
        for gb in batches[W:]:
            gb.reset()
        torch.cuda.synchronize()
        sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        ts = time.perf_counter()
        for k, gb in enumerate(batches[W:]):
            sev[k][0].record(stream)
            gb.rollout()
            sev[k][1].record(stream)
        torch.cuda.synchronize()
        el_s = time.perf_counter() - ts
        trans_s = sum(int(gb.steps.sum().item()) for gb in batches[W:])
        overlapped_ms = float(np.mean(kernel_ms))
        kernel_ms = [a.elapsed_time(b) for a, b in sev]
        serial = {"value_rank0": trans_s / el_s, "ms_per_step": el_s / K * 1e3,
                  "same_transitions": trans_s == trans_rank,
                  "overlapped_launch_avg_ms": overlapped_ms}
    # the launch lasts as long as its longest game (one wave per game, latency-bound)
    steps_max = float(np.mean([int(gb.steps.max().item()) for gb in batches[W:]]))
    errs = sum(int((gb.errors() != 0).sum().item()) for gb in batches[W:])
    unfinished = sum(int((~gb.terminal()).sum().item()) for gb in batches[W:])

    # End to end: the same K batches re-initialised (k_init: CPython seeding + deal)
    # and rolled out, init inside the timed region.
    ie = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for k, gb in enumerate(batches[W:]):
        ie[k][0].record(stream)
        gb.reset()
        ie[k][1].record(stream)
        gb.rollout()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed_e2e = time.perf_counter() - t1
    init_ms = float(np.mean([a.elapsed_time(b) for a, b in ie]))

    t = torch.tensor([elapsed, float(trans_rank), float(errs), float(unfinished), elapsed_e2e],
                     dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, elapsed_e2e = float(tmax[0]), float(tmax[4])
    trans_all, errs_all, unfinished_all = float(t[1]), int(t[2]), int(t[3])

    if rank == 0:
        per_launch_trans = trans_rank / K
        avg_ms = float(np.mean(kernel_ms))
        alg_bytes = per_launch_trans * 2 * L.GAME_BYTES
        achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
        traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
        n_gpus = min(world, max(1, n_dev))
        out = {
            "metric": "Option.carry_out steps/sec (whole node), 6-player batched self-play",
            "value": trans_all / elapsed,
            "unit": "carry_out transitions/s",
            "n_gpus": n_gpus,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: seeded preset games (run_utils.create_game), CPython-MT19937 random policy; "
                    "k_rollout_u is bit-exact with the reference per seed (tests/test_gpu_parity.py)",
            "config": {"workload": "config2: %d preset 6-player games per GPU, uniform random policy to terminal"
                                   % B, "games_per_gpu": B, "games_per_block": args.games_per_block,
                       "rng": "per-game CPython MT19937 (parity mode)", "parallelism": "dp%d" % world},
            "transitions_per_step": trans_all / K,
            "lane_errors": errs_all,
            "unfinished_lanes": unfinished_all,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": KERNEL if args.games_per_block <= 0 else "k_rollout (lanes)",
                         "kernel_avg_ms": avg_ms,
                         "alg_bytes_per_launch": alg_bytes,
                         "alg_bytes_per_transition": 2 * L.GAME_BYTES,
                         "measured_gbs": (traffic / (avg_ms * 1e-3) / 1e9) if traffic else None,
                         "issue": issue_roofline(pmc.get("sq") if pmc else None, per_launch_trans, avg_ms),
                         "latency": {"bound": "per-wave step latency x longest game",
                                     "steps_mean": per_launch_trans / B, "steps_max_mean_per_launch": steps_max,
                                     "us_per_step_longest_game": avg_ms * 1e3 / steps_max,
                                     "mean_over_max": per_launch_trans / B / steps_max},
                         "pmc": pmc},
            "streams": {"n": S, "one_stream": serial,
                        "note": "K batches launched round-robin on n HIP streams (n = 1: one after another); "
                                "roofline from one launch running alone"},
            "e2e": {"games_per_s": world * B * K / elapsed_e2e, "transitions_per_s": trans_all / elapsed_e2e,
                    "init_ms_per_batch": init_ms,
                    "note": "k_init (CPython init_by_array seeding + preset deal) inside the timed region"},
        }
        if folded:
            out["folded"] = True
            out["ranks"] = world
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.py_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
