"""Benchmark: Option.carry_out transitions/s, batched 6-player self-play.

Workload (BASELINE.json configs[1], "config 2"): per GPU, 4096 preset
6-player games (run_utils.create_game) played by the uniform random policy
to terminal.  One bench step = one launch of the fused rollout kernel
(k_rollout_u) over a fresh batch of 4096 games already resident in HBM
(initialised, untimed, before the timed region); seeds are disjoint across
steps and ranks (seed = base + (step * world + rank) * B + lane), so N GPUs
play N x 4096 independent games per step (weak scaling, no data-path
collective).  The K steps are launched round-robin on `--streams` HIP
streams (default 3, warmed before the timed region), so up to
`config.games_in_flight` = streams x 4096 games are resident at once: a
launch lasts as long as its longest game, and the next batches' games take
the SIMD slots the finished games free
(tests/test_gpu_parity.py::test_gpu_rollout_streams_overlap checks
overlapped batches equal batches run alone).  `value_one_batch` replays the
same K batches one after another (one batch resident at a time).

Prints ONE JSON line on rank 0.  `value` = carry_out transitions of all ranks
/ max-over-ranks wall time of the K timed steps.

* `roofline` prices one k_rollout_u launch running alone (the one-stream
  replay; the PMC children run with --streams 1).  The kernel keeps each game
  in LDS and is bound by instruction issue and per-wave latency, not HBM, so
  `bound` is "salu-issue": `achieved` = scalar instructions issued per second
  (SQ_INSTS_SALU from an in-run rocprofv3 --pmc pass over a short child run
  of this script) against the CU's one scalar issue per clock (`peak`,
  256 CU x 2.4 GHz), i.e. `frac` = SALU floor / kernel time;
  `wait_any_frac` (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and `busy_frac` (mean / max
  game length: one wave runs one game, so a launch lasts as long as its
  longest game) complete the latency model.  `hbm_notional` keeps SURVEY
  §8(d)'s HBM figure (2 x CIT_GAME_BYTES algorithmic bytes per transition
  over the kernel time, against 8 TB/s) and `measured_frac` the counter
  bytes (FETCH_SIZE + WRITE_SIZE, gfx950 FETCH half-count corrected) over the
  kernel time against the same peak.  Without the counters (N > 1, or
  --no-pmc) `bound` falls back to the notional HBM figure.
* `cpu_baseline` times the build's C++ CPU restatement (the same engine
  headers compiled with g++, build/libcitadels_hostcheck.so) on 1 host core
  and on all the cores this process may use, on rank 0 at N = 1, with nproc
  and the lscpu model; the pure-Python oracle (oracle/) is a secondary
  figure and the reference's own Python is quoted from BASELINE.md (measured
  in the survey container; it cannot travel to the GPU box).
* `e2e` adds the init: the same K batches re-initialised (k_mt_seed_cpython +
  k_init) and rolled out, init + rollout of batch k on stream k % streams, so
  the next batch's seeding overlaps the previous batches' rollouts.
* `cfr_configs` (default on; --no-cfr to skip) measures BASELINE configs 3-5,
  the MCCFR workloads, each a dict with its own value / unit, a roofline and
  a C++ CPU baseline (the same search headers built for the host,
  cith_cfr_timed, 1 core and all usable cores).  The search kernels are
  latency-bound (one wave per tree, a serial search), so `roofline` is the
  issue / latency model from in-run counters (four rocprofv3 --pmc passes
  over one `--pmc-child` run of the three workloads at small sizes, whose
  kernels are distinct): SALU floor over the search time, wait fraction,
  SALU / VALU / LDS / VMEM instructions and counter traffic per carry_out;
  `hbm_notional` keeps SURVEY §8(d)'s bytes per child created:
    3: 1024 positions per GPU, one cfr_train(200) decision each (no NN)
    4: 4096 positions over the job (4096 / N per GPU), cfr_pred(200, depth 10)
       with ValueOnlyNN(418, 512) weights from torch.manual_seed(0), one
       launch (k_cfr_pred_fused: each tree evaluates its leaves in its kernel)
    5: --cfg5-trees simulate_game trees per GPU at cfr_train(--cfg5-iters)
       (default 200000, the reference's own setting) through the tree queue,
       targets pooled with the RCCL all-gather; `value` = --cfg5-rounds data
       rounds through one cross-round queue (train_from_scratch's loop),
       `value_one_batch` = one round alone
  `4@512` and `5@960` run configs 4 and 5 at the per-rank shard of the 8-GPU
  job (4096 / 8 positions; train_from_scratch's --games-per-gpu trees).
  Config 3's `value` runs consecutive batches on --cfr-streams HIP streams
  (a continuous self-play loop, as config 2); `value_one_batch` is one batch
  at a time.
* `--config 3|4|5` makes that config the headline line instead (used for the
  PMC children and for A/B runs).
"""
import argparse
import ctypes as C
import glob
import csv
import json
import multiprocessing as mp
import os
import platform
import shutil
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
SALU_PEAK = N_CU * CLOCK_HZ  # one scalar instruction per clock per CU
BASE_SEED = 1_000_000_000
CFR_SEED = 30_000_000        # configs 3-5: positions / trees seeded from here (tools/bench_selfplay.py)
KERNELS = {2: "k_rollout_u", 3: "k_cfr_decide", 4: "k_cfr_pred_fused", 5: "k_cfr_train_slice"}
SEARCH_KERNELS = ("k_cfr_decide", "k_cfr_pred_fused", "k_cfr_train_slice", "k_cfr_pred_step")
# The reference's own Python, BASELINE.md §2 config 1 (survey container, 8-core Xeon).
REF_PY = {"1_core": 12301, "8_procs": 83869, "unit": "carry_out transitions/s",
          "where": "survey container (BASELINE.md), not this box"}
SQ_SET = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
          "SQ_BUSY_CYCLES", "SQ_INSTS_SMEM"]
MLP_FLOP_PER_ROW = 2 * (418 * 512 + 512 * 256 + 256 * 128 + 128 * 6)   # ValueOnlyNN(418, 512), BN folded
FP32_MATRIX_PEAK_TF = 157.3   # v_mfma_f32_16x16x4_f32 (MI355X_MICROARCH.md)
MLP_ROWS = 4096               # cfr_pred's rounds mode evaluates one leaf row per suspended tree (config 4: 4096)
MLP_KERNELS = ("k_mlp_layer", "k_mlp_head")
LINE_MAX_BYTES = 8192         # the stdout line the driver parses (round 5's 23 KB line was not parsed)


def _r(x, sig=4):
    """Floats to `sig` significant digits, recursively (the compact line)."""
    if isinstance(x, float):
        if x != x or x in (float("inf"), float("-inf")):
            return None
        return float("%.*g" % (sig, x))
    if isinstance(x, dict):
        return {k: _r(v, sig) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_r(v, sig) for v in x]
    return x


def _pick(d, *keys):
    d = d or {}
    return {k: d.get(k) for k in keys if d.get(k) is not None}


def compact_line(out, detail_path):
    """The one stdout line: the contract's fields, the headline roofline and CPU
    baseline, and per CFR leg its value, one-batch value, roofline fraction,
    traffic over §8(d)'s bytes and CPU baseline.  Everything else (counter
    passes, traces, notes, per-rep figures) stays in the full object written to
    `detail_path`."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "value_one_batch", "mode", "lane_errors", "unfinished_lanes", "folded",
            "ranks")
    line = {k: out[k] for k in keep if k in out}
    cfg = out.get("config") or {}
    line["config"] = _pick(cfg, "workload", "games_per_batch", "streams", "games_in_flight", "parallelism")
    roof = out.get("roofline") or {}
    line["roofline"] = _pick(roof, "bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_avg_ms",
                             "kernel_avg_ms_source", "traffic_over_alg")
    if roof.get("issue_bound"):
        line["roofline"]["issue_bound"] = _pick(roof["issue_bound"], "bound", "frac", "salu_per_transition",
                                                "wait_any_frac")
    if roof.get("timed_mode"):
        line["roofline"]["timed_mode_ms_per_step"] = roof["timed_mode"].get("ms_per_step")
    cpu = out.get("cpu_baseline")
    line["cpu_baseline"] = None if cpu is None else _pick(cpu, "value", "unit", "cores", "kind", "sample", "one_core",
                                                          "cpu_model", "error")
    if out.get("e2e"):
        line["e2e_transitions_per_s"] = out["e2e"].get("transitions_per_s")
    if out.get("cfr") is not None:          # --config 3|4|5 headline
        line["cfr"] = _cfr_compact(out["cfr"])
    legs = out.get("cfr_configs")
    if legs:
        line["cfr_configs"] = {k: (_cfr_compact(v) if isinstance(v, dict) and "value" in v else
                                   {"error": str((v or {}).get("error", v))[:160]} if isinstance(v, dict) else
                                   str(v)[:160]) for k, v in legs.items()}
    if out.get("mlp"):
        line["mlp"] = _pick(out["mlp"], "kernel", "rows", "tflops", "peak", "frac", "kernel_ms", "kernel_ms_source",
                            "error")
    line["detail"] = detail_path
    return _r(line)


def _cfr_compact(c):
    roof = c.get("roofline") or {}
    issue = roof.get("issue") or {}
    out = _pick(c, "value", "value_one_batch", "unit", "per_gpu")
    out["roofline"] = _pick(roof, "bound", "frac", "kernel", "kernel_avg_ms", "kernel_launches", "kernel_ms_source")
    if roof.get("traffic_over_alg") is not None or issue.get("traffic_over_alg") is not None:
        out["roofline"]["traffic_over_alg"] = roof.get("traffic_over_alg", issue.get("traffic_over_alg"))
    if issue.get("salu_per_carry_out") is not None:
        out["roofline"]["salu_per_carry_out"] = issue["salu_per_carry_out"]
    hn = roof.get("hbm_notional") or {}
    if hn.get("frac") is not None:
        out["roofline"]["hbm_notional_frac"] = hn["frac"]
    cpu = c.get("cpu_baseline")
    if cpu:
        out["cpu_baseline"] = _pick(cpu, "value", "one_core", "cores", "error")
    if c.get("rounds"):
        out["rounds"] = _pick(c["rounds"], "value", "rounds", "trees_per_round", "seconds", "loop")
    return out


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


def _hostlib():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import hostcheck
    return hostcheck.lib()


def cpu_baseline(seconds, py_seconds):
    """the build's C++ CPU restatement on 1 core and on all usable
    cores, plus the Python oracle (secondary)."""
    lib = _hostlib()
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


def cfr_cpu_baseline(config, iters, seconds, node_cap, edge_cap, weights=None):
    """The C++ restatement of the MCCFR workloads (cith_cfr_timed, the search
    headers built for the host) on 1 core and on all usable cores."""
    lib = _hostlib()
    f = lib.cith_cfr_timed
    f.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_double, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                  C.c_void_p, C.c_void_p, C.c_void_p]
    f.restype = C.c_int
    arr = None
    if weights is not None:
        ws = [np.ascontiguousarray(w, np.float32) for w in weights]
        arr = (C.c_void_p * 8)(*[w.ctypes.data for w in ws])
    threads = host_threads()
    legs = {}
    for name, th in (("1_core", 1), ("all_cores", threads)):
        d, c, e, w = C.c_longlong(), C.c_longlong(), C.c_longlong(), C.c_double()
        rc = f(config, iters, C.c_uint64(CFR_SEED + 50_000_000), C.c_double(seconds), th, node_cap, edge_cap, arr,
               C.byref(d), C.byref(c), C.byref(e), C.byref(w))
        if rc != 0:
            raise RuntimeError("cith_cfr_timed(%d) returned %d" % (config, rc))
        legs[name] = {"value": d.value / w.value, "threads": th, "units": d.value, "carry_outs": c.value,
                      "carry_out_per_s": c.value / w.value, "error_lanes": e.value, "wall_s": w.value}
    a = legs["all_cores"]
    unit = "trees/s" if config == 5 else "decisions/s"
    return {"value": a["value"], "unit": unit, "cores": a["threads"], "kind": "port",
            "impl": "cpp-restatement: the search headers (csrc/cit_cfr.h, cit_engine.h) built with g++ -O3 for the "
                    "host (cith_cfr_timed), one tree per thread" + (", host fp32 value net" if config == 4 else ""),
            "sample": "%d %s on %d threads x %.0f s, %d on 1 core x %.0f s" % (
                a["units"], "trees" if config == 5 else "decisions", a["threads"], seconds, legs["1_core"]["units"],
                seconds),
            "one_core": legs["1_core"]["value"], "legs": legs, "nproc": os.cpu_count(), "usable_cores": threads,
            "cpu_model": cpu_model()}


def _rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def _run_profiled(prof_args, child, outdir, timeout_s):
    """rocprofv3 `prof_args` over `child` (its own process group, killed on
    timeout), output under outdir.  Returns the log's path; raises on failure."""
    os.makedirs(outdir, exist_ok=True)
    # (a child must not overwrite the parent's full-object file)
    child = child + ["--full-out", os.path.join(outdir, "child_full.json")]
    cmd = ["rocprofv3"] + prof_args + ["--output-format", "csv", "-d", outdir, "-o", "run", "--"] + child
    env = dict(os.environ, TMPDIR="/tmp")
    logp = os.path.join(outdir, "log.txt")
    t0 = time.perf_counter()
    with open(logp, "w") as log:
        p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
        rc = None
        while rc is None:
            try:
                rc = p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                el = time.perf_counter() - t0
                if el > timeout_s:
                    os.killpg(p.pid, signal.SIGKILL)
                    p.wait()
                    raise RuntimeError("rocprofv3 %s timed out" % " ".join(prof_args))
                _progress("rocprofv3 %s child running (%.0f s)" % (" ".join(prof_args)[:60], el))
    _progress("rocprofv3 %s child done (%.0f s)" % (" ".join(prof_args)[:60], time.perf_counter() - t0))
    if rc != 0:
        raise RuntimeError("rocprofv3 %s exited %d" % (" ".join(prof_args), rc))
    return logp


def _progress(msg):
    """A progress line on stderr (long profiler children otherwise leave a
    run silent for minutes)."""
    print("bench: " + msg, file=sys.stderr, flush=True)


def _child_line(logp):
    with open(logp) as f:
        lines = [ln for ln in f if ln.startswith("{\"pmc_child\"")]
    if not lines:
        raise RuntimeError("no child line in the rocprofv3 output")
    return json.loads(lines[-1])


def _by_leg(per_kernel, child):
    """{kernel: {dispatch id: value}} -> {leg key: [values of its launches]}:
    the child runs PMC_CHILD_LEGS in order and reports each leg's launches of
    every search kernel (a config-5 leg searches through the tree queue's
    k_cfr_train_slice, or through k_cfr_decide when its trees fit at once; an
    overflowed tree is searched again by k_cfr_decide), so a kernel's
    dispatches, in dispatch order, go to the legs in turn."""
    taken, out = {}, {}
    for key, c, _ in PMC_CHILD_LEGS:
        launches = child[key]["launches"]
        if not isinstance(launches, dict):          # (an older child line: its own kernel only)
            launches = {KERNELS[c]: launches}
        vals = []
        for k, n in launches.items():
            ids = sorted(per_kernel.get(k, {}))
            mine = ids[taken.get(k, 0):taken.get(k, 0) + int(n)]
            taken[k] = taken.get(k, 0) + int(n)
            vals += [per_kernel[k][i] for i in mine]
        out[key] = vals
    return out


def _pmc_pass(counters, outdir, config=2, timeout_s=150, cfr_child=False):
    """One rocprofv3 --pmc pass over a short child run of this script (its own
    process group, killed on timeout).  Config 2: {counter: mean per launch of
    k_rollout_u}.  cfr_child: the child runs configs 3 / 4 / 5 once each
    (--pmc-child) and the result is {kernel: {counter: sum over its launches,
    "_launches": n}, "_child": the child's JSON line}.  Raises on failure."""
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-pmc"]
    if cfr_child:
        child += ["--pmc-child"]
    else:
        child += ["--config", str(config), "--no-cfr"]
        child += ["--steps", "2", "--warmup", "1", "--streams", "1"] if config == 2 else [
            "--cfr-reps", "1", "--cfg5-reps", "1", "--cfr-streams", "1"]
    logp = _run_profiled(["--pmc"] + counters, child, outdir, timeout_s)
    rows = _rows(os.path.join(outdir, "**", "*counter_collection.csv"))
    if cfr_child:
        child = _child_line(logp)
        per_kernel = {}
        for r in rows:
            k = next((k for k in SEARCH_KERNELS if k in r.get("Kernel_Name", "")), None)
            if k is not None and "Dispatch_Id" in r:
                d = per_kernel.setdefault(k, {}).setdefault(int(r["Dispatch_Id"]), {})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        out = {}
        for key, launches in _by_leg(per_kernel, child).items():
            tot = {}
            for d in launches:
                for name, v in d.items():
                    tot[name] = tot.get(name, 0.0) + v
            if tot:
                tot["_launches"] = len(launches)
                out[key] = tot
        if not out:
            raise RuntimeError("no search-kernel rows in the rocprofv3 output")
        out["_child"] = child
        return out
    kernel = KERNELS[config]
    per = {}
    for r in rows:
        if kernel in r.get("Kernel_Name", ""):
            per.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id", "0"), 0.0)
            per[r["Counter_Name"]][r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
    if not per:
        raise RuntimeError("no %s rows in the rocprofv3 output" % kernel)
    out = {k: sum(v.values()) / len(v) for k, v in per.items()}
    out["_launches"] = max(len(v) for v in per.values())
    return out


def trace_in_run(args, timeout_s=300):
    """rocprofv3 --kernel-trace --stats over a child run of this script's
    config-2 workload with every launch alone (--streams 1, the same --steps /
    --warmup): {calls, avg_ms, min_ms, max_ms} of k_rollout_u and the stats
    CSV's path.  The roofline is priced on this duration (the profiler's
    kernel begin / end), not on HIP events around the launch."""
    outdir = tempfile.mkdtemp(prefix="bench_trace_", dir="/tmp")
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-pmc", "--no-cfr",
             "--config", "2", "--streams", "1", "--steps", str(args.steps), "--warmup", str(args.warmup),
             "--batch", str(args.batch)]
    try:
        _run_profiled(["--kernel-trace", "--stats"], child, outdir, timeout_s)
        paths = glob.glob(os.path.join(outdir, "**", "*kernel_stats.csv"), recursive=True)
        rows = _rows(os.path.join(outdir, "**", "*kernel_stats.csv"))
        row = next(r for r in rows if KERNELS[2] in r["Name"])
        return {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) * 1e-6,
                "min_ms": float(row["MinNs"]) * 1e-6, "max_ms": float(row["MaxNs"]) * 1e-6,
                "stats_csv": paths[0] if paths else None,
                "command": "rocprofv3 --kernel-trace --stats -- python bench.py --config 2 --streams 1 --steps %d "
                           "--warmup %d --no-cfr --no-pmc --no-cpu-baseline" % (args.steps, args.warmup)}
    except Exception as e:  # a missing profiler must not cost the bench line
        return {"error": str(e)[:300]}


def pmc_in_run(config=2):
    """Three --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ set), each its own child run."""
    base = tempfile.mkdtemp(prefix="bench_pmc_", dir="/tmp")
    out = {"source": "in-run rocprofv3 --pmc, 3 passes over `bench.py --config %d` children" % config,
           "kernel": KERNELS[config]}
    try:
        f = _pmc_pass(["FETCH_SIZE"], os.path.join(base, "fetch"), config)["FETCH_SIZE"]
        w = _pmc_pass(["WRITE_SIZE"], os.path.join(base, "write"), config)["WRITE_SIZE"]
        out["fetch_size_kib"] = f
        out["write_size_kib"] = w
        out["hbm_bytes_per_launch"] = 2 * 1024 * f + 1024 * w
        out["sq"] = _pmc_pass(SQ_SET, os.path.join(base, "sq"), config)
    except Exception as e:  # a missing profiler must not cost the bench line
        out["error"] = str(e)[:300]
    return out


# Counter passes over one --pmc-child run of the three search workloads (their
# kernels are distinct, so one child serves configs 3, 4 and 5).
CFR_PMC_PASSES = (["FETCH_SIZE"], ["WRITE_SIZE"], SQ_SET, ["SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"])
# The --pmc-child run's legs, in order: (key, config, positions / trees).  Config 5
# runs at its bench size: fewer trees fit in HBM at once and would search in
# k_cfr_decide (simulate_games without the queue), not in the queue's
# k_cfr_train_slice.  "4@512" is config 4's per-rank shard of the 8-GPU job.
PMC_CHILD_LEGS = (("3", 3, 1024), ("4@512", 4, 512), ("4", 4, 4096), ("5", 5, 1920), ("5@960", 5, 960))


def pmc_in_run_cfr():
    """Four --pmc passes over `bench.py --pmc-child` (PMC_CHILD_LEGS once each,
    no warm-up).  Returns {leg key: {counter: total over the leg's launches,
    "carry_outs": the child's carry_outs, "search_ms": its search time}}."""
    base = tempfile.mkdtemp(prefix="bench_pmc_cfr_", dir="/tmp")
    out = {}
    try:
        for i, ctrs in enumerate(CFR_PMC_PASSES):
            r = _pmc_pass(ctrs, os.path.join(base, "p%d" % i), cfr_child=True, timeout_s=240)
            child = r.pop("_child")
            for key, c, n in PMC_CHILD_LEGS:
                d = out.setdefault(key, {"kernel": KERNELS[c], "source": "in-run rocprofv3 --pmc, %d passes over one "
                                         "`bench.py --pmc-child` run (%d %s)" % (len(CFR_PMC_PASSES), n,
                                                                           "trees" if c == 5 else "positions")})
                d.update(r.get(key, {}))
                d["carry_outs_pass%d" % i] = child[key]["carry_outs"]
                d["search_ms_pass%d" % i] = child[key]["search_ms"]
                d["carry_outs"] = child[key]["carry_outs"]
    except Exception as e:  # a missing profiler must not cost the bench line
        out["error"] = str(e)[:300]
    return out


def trace_in_run_cfr(timeout_s=300):
    """rocprofv3 --kernel-trace --stats over one `bench.py --pmc-child` run (the
    counter passes' own workload and seeds): per leg, its search kernel's
    launches and their durations (the profiler's kernel begin / end), and the
    value-net kernels of the child's MLP leg.  The CFR rooflines are priced on
    these durations."""
    outdir = tempfile.mkdtemp(prefix="bench_cfrtrace_", dir="/tmp")
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-pmc", "--pmc-child"]
    try:
        logp = _run_profiled(["--kernel-trace", "--stats"], child, outdir, timeout_s)
        child_line = _child_line(logp)
        rows = _rows(os.path.join(outdir, "**", "*kernel_trace.csv"))
        per_kernel, mlp = {}, {}
        for r in rows:
            name = r.get("Kernel_Name", "")
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            k = next((k for k in SEARCH_KERNELS if k in name), None)
            if k is not None:
                per_kernel.setdefault(k, {})[int(r["Dispatch_Id"])] = dur
            m = next((m for m in MLP_KERNELS if m in name), None)
            if m is not None:
                mlp.setdefault(m, []).append(dur)
        out = {}
        for key, durs in _by_leg(per_kernel, child_line).items():
            if durs:
                out[key] = {"launches": len(durs), "kernel_ms_total": float(sum(durs)),
                            "kernel_avg_ms": float(sum(durs) / len(durs)), "carry_outs": child_line[key]["carry_outs"],
                            "kernels": child_line[key]["launches"]}
        if mlp and child_line.get("mlp"):
            calls = int(child_line["mlp"]["calls"])
            out["mlp"] = {"calls": calls, "rows": child_line["mlp"]["rows"],
                          "kernel_ms_per_call": sum(sum(v) for v in mlp.values()) / max(1, calls),
                          "per_kernel_avg_ms": {k: sum(v) / len(v) for k, v in mlp.items()}}
        out["_stats_csv"] = (glob.glob(os.path.join(outdir, "**", "*kernel_stats.csv"), recursive=True) or [None])[0]
        out["_command"] = "rocprofv3 --kernel-trace --stats -- python bench.py --pmc-child --no-pmc --no-cpu-baseline"
        return out
    except Exception as e:  # a missing profiler must not cost the bench line
        return {"error": str(e)[:300]}


def search_roofline(pmc, alg_bytes_per_carry, timed_ms, timed_carry, trace=None):
    """The latency / issue model of a search kernel from its in-run counters
    (totals over the child's launches, priced per carry_out; the child runs
    the timed rep's seeds, unwarmed and serialised by the profiler, so its own
    wall time is not the kernel's): SALU instructions per carry_out x the
    timed rep's carry_outs as the SALU floor against the timed search, wait
    fraction, VMEM instructions and counter traffic per carry_out against
    SURVEY §8(d)'s algorithmic bytes."""
    if not pmc or "SQ_INSTS_SALU" not in pmc:
        return None
    carry = float(pmc.get("carry_outs_pass2", pmc["carry_outs"]))    # the SQ pass's own run
    salu = pmc["SQ_INSTS_SALU"]
    salu_timed = salu / carry * timed_carry
    salu_floor_ms = salu_timed / SALU_PEAK * 1e3
    out = {"salu_per_carry_out": salu / carry, "valu_per_carry_out": pmc.get("SQ_INSTS_VALU", 0.0) / carry,
           "lds_per_carry_out": pmc.get("SQ_INSTS_LDS", 0.0) / carry,
           "smem_per_carry_out": pmc.get("SQ_INSTS_SMEM", 0.0) / carry,
           "salu_floor_ms": salu_floor_ms, "search_ms": timed_ms,
           "salu_frac": salu_floor_ms / timed_ms if timed_ms else None,
           "salu_inst_per_s": salu_timed / (timed_ms * 1e-3) if timed_ms else None,
           "child_carry_outs": carry, "child_search_ms": float(pmc.get("search_ms_pass2") or 0.0),
           "launches": pmc.get("_launches")}
    if pmc.get("SQ_WAVE_CYCLES"):
        out["wait_any_frac"] = pmc.get("SQ_WAIT_ANY", 0.0) / pmc["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VMEM_RD" in pmc:
        c3 = float(pmc.get("carry_outs_pass3", carry))
        out["vmem_rd_per_carry_out"] = pmc["SQ_INSTS_VMEM_RD"] / c3
        out["vmem_wr_per_carry_out"] = pmc.get("SQ_INSTS_VMEM_WR", 0.0) / c3
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        c0, c1 = float(pmc.get("carry_outs_pass0", carry)), float(pmc.get("carry_outs_pass1", carry))
        per = 2 * 1024 * pmc["FETCH_SIZE"] / c0 + 1024 * pmc["WRITE_SIZE"] / c1
        out["traffic_bytes_per_carry_out"] = per
        out["traffic_over_alg"] = per / alg_bytes_per_carry if alg_bytes_per_carry else None
    if trace and trace.get("kernel_ms_total"):
        # priced on the kernel trace of the same workload (the counter child's seeds, so its carry_outs): the
        # SALU floor of its carry_outs over the profiler's summed kernel durations
        floor_ms = salu / carry * float(trace["carry_outs"]) / SALU_PEAK * 1e3
        out["salu_frac_timed_search"] = out["salu_frac"]
        out["salu_frac"] = floor_ms / trace["kernel_ms_total"]
        out["kernel_ms_total"] = trace["kernel_ms_total"]
        out["kernel_avg_ms"] = trace["kernel_avg_ms"]
        out["kernel_launches"] = trace["launches"]
        out["salu_inst_per_s"] = salu / carry * float(trace["carry_outs"]) / (trace["kernel_ms_total"] * 1e-3)
    return out


def issue_roofline(sq, units_per_launch, kernel_ms, unit="transition"):
    """What bounds a latency-bound kernel: instruction issue, from the SQ
    counters (per-wave instruction counts; SQ_*_CYCLES used only as a ratio)."""
    if not sq or "SQ_INSTS_SALU" not in sq:
        return None
    salu, valu, lds = sq["SQ_INSTS_SALU"], sq.get("SQ_INSTS_VALU", 0.0), sq.get("SQ_INSTS_LDS", 0.0)
    salu_floor_ms = salu / SALU_PEAK * 1e3                              # 1 scalar issue / clk / CU
    valu_floor_ms = valu * 2 / (N_CU * SIMD_PER_CU * CLOCK_HZ) * 1e3    # wave64 on SIMD32: 2 clk
    out = {"salu_per_%s" % unit: salu / units_per_launch, "valu_per_%s" % unit: valu / units_per_launch,
           "lds_per_%s" % unit: lds / units_per_launch, "salu_floor_ms": salu_floor_ms,
           "valu_floor_ms": valu_floor_ms, "salu_frac": salu_floor_ms / kernel_ms,
           "salu_inst_per_s": salu / (kernel_ms * 1e-3),
           "model": "SALU floor = SQ_INSTS_SALU / (256 CU x 2.4 GHz x 1 SALU/clk); frac = floor / kernel time"}
    if sq.get("SQ_WAVE_CYCLES"):
        out["wait_any_frac"] = sq.get("SQ_WAIT_ANY", 0.0) / sq["SQ_WAVE_CYCLES"]
    return out


def _barrier(world):
    if world > 1:
        dist.barrier()


def _reduce(vals, world, dev, maxes=()):
    """SUM over ranks, except the indices in `maxes` (MAX)."""
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        for i in maxes:
            t[i] = tmax[i]
    return [float(x) for x in t]


def run_rollout(args, world, rank, dev, n_dev, pmc):
    """Config 2: the headline.  Returns the bench line (rank 0) or None."""
    from citadels_self_play_amd import layout as L
    from citadels_self_play_amd.engine import GameBatch, side_streams

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
    streams = [stream] if S == 1 else side_streams(dev, S)     # (one pool for every leg: engine.side_streams)
    if S > 1:
        # A stream's first launches set up its hardware queue: warm every stream
        # with a small init + rollout of its own (untimed, seeds outside the timed ones).
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                for _ in range(2):
                    GameBatch(np.arange(BASE_SEED - (i + 1) * 256, BASE_SEED - i * 256), preset=True, device=dev,
                              games_per_block=args.games_per_block).rollout()
        torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    _barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, gb in enumerate(batches[W:]):
        st = streams[k % S]
        with torch.cuda.stream(st):
            evs[k][0].record(st)
            gb.rollout()
            evs[k][1].record(st)
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = time.perf_counter() - t0

    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    trans_rank = sum(int(gb.steps.sum().item()) for gb in batches[W:])
    overlapped_ms = float(np.mean(kernel_ms))
    queue = None
    if args.queue:
        queue = _rollout_queue_run(args, world, rank, dev, B, K, trans_rank)
    # One batch resident at a time: the same K batches re-initialised (untimed)
    # and replayed one after another on one stream; the roofline prices these
    # launches (a kernel running alone).
    el_s, trans_s = elapsed, trans_rank
    if S > 1:
        for gb in batches[W:]:
            gb.reset()
        torch.cuda.synchronize()
        sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        _barrier(world)
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for k, gb in enumerate(batches[W:]):
            sev[k][0].record(stream)
            gb.rollout()
            sev[k][1].record(stream)
        torch.cuda.synchronize()
        _barrier(world)
        el_s = time.perf_counter() - ts
        trans_s = sum(int(gb.steps.sum().item()) for gb in batches[W:])
        kernel_ms = [a.elapsed_time(b) for a, b in sev]
    # the launch lasts as long as its longest game (one wave per game, latency-bound)
    steps_max = float(np.mean([int(gb.steps.max().item()) for gb in batches[W:]]))
    errs = sum(int((gb.errors() != 0).sum().item()) for gb in batches[W:])
    unfinished = sum(int((~gb.terminal()).sum().item()) for gb in batches[W:])

    # End to end: the same K batches re-initialised (k_mt_seed_cpython + k_init)
    # and rolled out, init inside the timed region; init + rollout of batch k
    # on stream k % S, so the next batches' seeding overlaps earlier rollouts.
    ie = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    _barrier(world)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for k, gb in enumerate(batches[W:]):
        st = streams[k % S]
        with torch.cuda.stream(st):
            ie[k][0].record(st)
            gb.reset()
            ie[k][1].record(st)
            gb.rollout()
    torch.cuda.synchronize()
    _barrier(world)
    elapsed_e2e = time.perf_counter() - t1
    init_ms = float(np.mean([a.elapsed_time(b) for a, b in ie]))
    trans_e2e = sum(int(gb.steps.sum().item()) for gb in batches[W:])

    elapsed, trans_all, errs_all, unfinished_all, elapsed_e2e, el_s, trans_s_all, trans_e2e_all = _reduce(
        [elapsed, trans_rank, errs, unfinished, elapsed_e2e, el_s, trans_s, trans_e2e], world, dev, maxes=(0, 4, 5))
    if rank != 0:
        return None
    per_launch_trans = trans_s / K
    events_ms = float(np.mean(kernel_ms))
    trace = (pmc or {}).get("trace") or {}
    # the kernel's own duration from the in-run kernel trace (every launch alone); HIP events otherwise
    avg_ms = trace["avg_ms"] if trace.get("avg_ms") else events_ms
    alg_bytes = per_launch_trans * 2 * L.GAME_BYTES
    hbm_achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    issue = issue_roofline(pmc.get("sq") if pmc else None, per_launch_trans, avg_ms)
    busy = per_launch_trans / B / steps_max
    hbm_notional = {"achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_achieved / HBM_PEAK_GBS,
                    "alg_bytes_per_launch": alg_bytes, "alg_bytes_per_transition": 2 * L.GAME_BYTES,
                    "model": "SURVEY §8(d): 2 x CIT_GAME_BYTES per transition over the kernel time (the row stays in "
                             "LDS, so these bytes never reach HBM)"}
    # the contract's roofline: SURVEY §8(d)'s algorithmic bytes over the kernel's own duration against HBM
    # peak, `traffic` the counter bytes per launch; what actually binds the kernel (scalar issue and the
    # per-wave latency chain: the row lives in LDS) is `issue_bound`
    roof = {"bound": "hbm", "achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": hbm_achieved / HBM_PEAK_GBS,
            "traffic_over_alg": (traffic / alg_bytes) if traffic else None}
    if issue is not None:
        roof["issue_bound"] = {"bound": "salu-issue", "achieved": issue["salu_inst_per_s"] / 1e9,
                               "peak": SALU_PEAK / 1e9, "unit": "G SALU inst/s", "frac": issue["salu_frac"],
                               "salu_per_transition": issue["salu_per_transition"],
                               "wait_any_frac": issue.get("wait_any_frac")}
    roof.update({
        "traffic": traffic, "kernel": KERNELS[2] if args.games_per_block <= 0 else "k_rollout (lanes)",
        "kernel_avg_ms": avg_ms, "launches": K,
        "kernel_avg_ms_source": "rocprofv3 --kernel-trace (in-run child, %d launches alone)" % trace["calls"]
        if trace.get("avg_ms") else "HIP events around each launch (one stream)",
        "kernel_avg_ms_events": events_ms, "trace": trace or None,
        "timed_mode": {"ms_per_step": elapsed / K * 1e3, "streams": S,
                       "hbm_notional_gbs": per_launch_trans * 2 * L.GAME_BYTES / (elapsed / K) / 1e9,
                       "note": "the headline's own clock: K launches on S streams overlapping, per step"},
        "wait_any_frac": issue.get("wait_any_frac") if issue else None, "busy_frac": busy,
        "hbm_notional": hbm_notional,
        "measured_gbs": (traffic / (avg_ms * 1e-3) / 1e9) if traffic else None,
        "measured_frac": (traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if traffic else None,
        "issue": issue,
        "latency": {"bound": "per-wave step latency x longest game",
                    "steps_mean": per_launch_trans / B, "steps_max_mean_per_launch": steps_max,
                    "us_per_step_longest_game": avg_ms * 1e3 / steps_max, "mean_over_max": busy},
        "pmc": pmc})
    n_gpus = min(world, max(1, n_dev))
    value, ms_step = trans_all / elapsed, elapsed / K * 1e3
    mode = "streams"
    if queue is not None:
        value, ms_step, mode = queue["value"], queue["ms_per_step"], "queue"
    return {
        "metric": "Option.carry_out steps/sec (whole node), 6-player batched self-play",
        "value": value,
        "unit": "carry_out transitions/s",
        "n_gpus": n_gpus,
        "steps": K,
        "warmup": W,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded preset games (run_utils.create_game), CPython-MT19937 random policy; "
                "k_rollout_u is bit-exact with the reference per seed (tests/test_gpu_parity.py)",
        "config": {"workload": "config2: %d preset 6-player games per batch, uniform random policy to terminal; "
                               "batches on %d HIP stream(s), up to %d games resident per GPU" % (B, S, S * B),
                   "games_per_batch": B, "streams": S, "games_in_flight": S * B,
                   "games_per_block": args.games_per_block,
                   "rng": "per-game CPython MT19937 (parity mode)", "parallelism": "dp%d" % world},
        "value_one_batch": trans_s_all / el_s,
        "transitions_per_step": trans_all / K,
        "lane_errors": errs_all,
        "unfinished_lanes": unfinished_all,
        "roofline": roof,
        "mode": mode,
        "queue": queue,
        "streams": {"n": S, "value": trans_all / elapsed, "one_batch": {"value": trans_s_all / el_s, "ms_per_step": el_s / K * 1e3,
                                          "same_transitions": trans_s_all == trans_all},
                    "overlapped_launch_avg_ms": overlapped_ms,
                    "note": "K batches launched round-robin on n HIP streams; one_batch replays them one after "
                            "another; the roofline is priced on one launch running alone"},
        "e2e": {"games_per_s": world * B * K / elapsed_e2e, "transitions_per_s": trans_e2e_all / elapsed_e2e,
                "init_ms_per_batch": init_ms, "streams": S,
                "note": "k_mt_seed_cpython + k_init inside the timed region, init + rollout of batch k on stream "
                        "k %% %d" % S},
    }


def _rollout_queue_run(args, world, rank, dev, B, K, trans_ref):
    """The K timed batches' games (the same seeds) as ONE work queue:
    cit_rollout_queue with as many one-wave workgroups as the GPU holds; a
    finished game's slot takes the next game at once.  Returns rank-local
    timing folded over ranks (max time, summed transitions)."""
    from citadels_self_play_amd.engine import GameBatch
    seeds = np.concatenate([np.arange(BASE_SEED + ((args.warmup + k) * world + rank) * B,
                                      BASE_SEED + ((args.warmup + k) * world + rank) * B + B) for k in range(K)])
    big = GameBatch(seeds, preset=True, device=dev)
    warm = GameBatch(np.arange(BASE_SEED - 8192, BASE_SEED), preset=True, device=dev)
    warm.rollout_queue()
    torch.cuda.synchronize()
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    _barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    big.rollout_queue()
    ev[1].record()
    torch.cuda.synchronize()
    _barrier(world)
    el = time.perf_counter() - t0
    trans = int(big.steps.sum().item())
    errs = int((big.errors() != 0).sum().item())
    el, trans_all, errs = _reduce([el, trans, errs], world, dev, maxes=(0,))
    return {"value": trans_all / el, "ms_per_step": el / K * 1e3, "kernel_ms": ev[0].elapsed_time(ev[1]),
            "games": int(len(seeds)) * world, "same_transitions_as_streams": trans == trans_ref,
            "lane_errors": int(errs),
            "note": "the K batches' %d games as one work queue (cit_rollout_queue, %d resident waves)"
                    % (len(seeds), 8 * 4 * torch.cuda.get_device_properties(dev).multi_processor_count)}


def _value_net(dev):
    from citadels_self_play_amd import models, selfplay
    torch.manual_seed(0)
    m = selfplay.broadcast_model(models.ValueOnlyNN(418, 512).to(dev).eval())
    return models.ValueNet(m, dev)


def run_cfr(config, args, world, rank, dev, pmc=None, cpu=True, per_gpu=None, warm_rep=True, n_reps=None,
            trace=None):
    """One of BASELINE configs 3-5 (tools/bench_selfplay.py's harness): median
    of `args.cfr_reps` timed reps after one warm-up.  `per_gpu` overrides the
    positions / trees per GPU (the per-rank shard of an 8-GPU config).  `pmc`:
    this config's entry of pmc_in_run_cfr.  Returns a dict (rank 0)."""
    from citadels_self_play_amd import layout as L
    from citadels_self_play_amd import selfplay
    from citadels_self_play_amd.engine import GameBatch, pool_caps
    iters = {3: 200, 4: 200, 5: args.cfg5_iters}[config]
    shard_leg = per_gpu is not None
    if per_gpu is None:
        per_gpu = {3: 1024, 4: max(1, 4096 // world), 5: args.cfg5_trees}[config]
    net = _value_net(dev) if config == 4 else None
    # one 4096-node block per tree either way; room enough that no config-3/4 tree
    # overflows into the (serial) retry
    node_cap = {3: 4096, 4: 4096}.get(config)
    reps = []
    stream = torch.cuda.current_stream()
    if n_reps is None:
        n_reps = args.cfg5_reps if config == 5 else args.cfr_reps
    for rep in range(0 if warm_rep else 1, 1 + n_reps):
        warm = rep == 0
        # config 5's warm-up: the timed rep's trees and node-pool caps at 2,000 iterations, so the
        # timed rep reuses the warm-up's cached arena (a one-time hipMalloc of up to ~230 GB, as the
        # first data round of a training run pays it) -- the search itself is the timed rep's own
        n = per_gpu
        it = iters if not (warm and config == 5) else min(iters, 2000)
        seeds = selfplay.shard(n * world, base_seed=CFR_SEED + rep * 1_000_000)
        if config in (3, 4):
            b = GameBatch(seeds, preset=True, device=dev)
            b.advance_random(0, 300)
            b.seed_numpy()
        torch.cuda.synchronize()
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        _barrier(world)
        t0 = time.perf_counter()
        ev[0].record(stream)
        rounds, n_targets = 0, 0
        if config == 3:
            chosen, stats = b.cfr_decide(it, node_cap=node_cap)
            term = b.terminal()
        elif config == 4:
            chosen, stats, rounds = b.cfr_pred(it, net, max_depth=10, node_cap=node_cap)
            term = b.terminal()
        else:
            nc5, ec5 = pool_caps(iters)
            b, stats, t = selfplay.simulate_games(
                seeds, it, node_cap=nc5, edge_cap=ec5,
                log=(lambda m: print(m, file=sys.stderr, flush=True)) if (rank == 0 and not warm) else None)
            f, v = selfplay.all_gather_targets(t["feat"], t["value"])
            n_targets = int(f.shape[0])
            term = t["terminal"]
        ev[1].record(stream)
        torch.cuda.synchronize()
        _barrier(world)
        el = time.perf_counter() - t0
        if warm:
            continue
        st = stats.to(dev).to(torch.float64)
        bad = ((st[:, 4] != 0) & ~term.to(dev)).sum()
        _, cls = selfplay.error_classes(stats, term)
        el_max, units, carry, nodes, edges, errs, terms, *ncls = _reduce(
            [el, st.shape[0], st[:, 3].sum(), st[:, 1].sum(), st[:, 2].sum(), bad, term.sum()] +
            [cls[k] for k in selfplay.ERROR_CLASSES], world, dev, maxes=(0,))
        reps.append({"seconds": el_max, "gpu_ms_rank0": ev[0].elapsed_time(ev[1]), "units": units,
                     "value": units / el_max, "carry_out_per_s": carry / el_max, "nodes": nodes, "edges": edges,
                     "error_lanes_nonterminal": int(errs), "terminal_positions": int(terms), "leaf_rounds": rounds,
                     "error_classes": {k: int(v) for k, v in zip(selfplay.ERROR_CLASSES, ncls)},
                     "pooled_targets": n_targets})
    # the reps' batches (config 5's one-round batch may hold its whole node arena) go before the next runs
    b = stats = t = term = st = None
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    streams = None
    if config == 3 and args.cfr_streams > 1:
        streams = _cfr_streams(args, world, rank, dev, iters, per_gpu, node_cap)
    rounds = None
    if config == 5 and args.cfg5_rounds > 1 and warm_rep:
        rounds = _cfg5_rounds(args, world, rank, dev, iters, per_gpu)
    if rank != 0:
        return None
    med = sorted(reps, key=lambda r: r["value"])[len(reps) // 2]
    S = L.GAME_BYTES
    # per child created 2S (row copy) + 2S (transition) + S (determinize) + 24 B per edge slot
    alg = med["nodes"] * 5 * S + 24.0 * med["edges"]
    ms = med["seconds"] * 1e3
    achieved = alg / world / med["seconds"] / 1e9          # per GPU
    carry_all = med["carry_out_per_s"] * med["seconds"]
    hbm_notional = {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                    "alg_bytes": alg, "alg_bytes_per_carry_out": alg / max(1.0, carry_all), "search_ms": ms,
                    "model": "SURVEY §8(d) CFR expand bytes: 5 x CIT_GAME_BYTES per node created + 24 B per edge "
                             "slot, over the search's wall time per GPU"}
    issue = search_roofline(pmc, alg / max(1.0, carry_all), ms, carry_all, trace=trace) if pmc else None
    if issue is not None and issue.get("salu_frac") is not None:
        roof = {"bound": "latency (salu-issue floor)", "achieved": issue["salu_inst_per_s"] / 1e9,
                "peak": SALU_PEAK / 1e9, "unit": "G SALU inst/s", "frac": issue["salu_frac"],
                "traffic_bytes_per_carry_out": issue.get("traffic_bytes_per_carry_out"),
                "traffic": issue.get("traffic_bytes_per_carry_out"),
                "traffic_over_alg": issue.get("traffic_over_alg"),
                "kernel_avg_ms": issue.get("kernel_avg_ms"), "kernel_launches": issue.get("kernel_launches"),
                "kernel_ms_source": ("rocprofv3 --kernel-trace of the counter child's workload (same seeds)"
                                     if issue.get("kernel_avg_ms") else "host wall clock of the timed search"),
                "model": "one wave per tree runs a serial search: the SALU floor (the counter run's "
                         "SQ_INSTS_SALU per carry_out x the traced run's carry_outs / (256 CU x 2.4 GHz)) over "
                         "the traced kernel time, with the wait fraction and VMEM instructions per carry_out; "
                         "hbm_notional keeps SURVEY §8(d)'s bytes"}
    else:
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                "note": "no SQ counters for this leg: SURVEY §8(d)'s notional HBM figure"}
    kern = "+".join(sorted((trace or {}).get("kernels") or {})) if isinstance((trace or {}).get("kernels"), dict) \
        else KERNELS[config]
    roof.update({"kernel": kern or KERNELS[config], "issue": issue, "hbm_notional": hbm_notional, "pmc": pmc,
                 "search_ms": ms})
    out = {"config": config, "workload": {
        3: "config3: %d positions per GPU (preset game + U[0,300] random steps), one cfr_train(200) decision each"
           % per_gpu,
        4: "config4: %d positions per GPU (%d over the job), cfr_pred(200, depth 10) + ValueOnlyNN(418,512) "
           "leaves (torch.manual_seed(0) weights)" % (per_gpu, per_gpu * world),
        5: "config5: %d simulate_game trees per GPU: create_a_random_game(100) -> cfr_train(%d) -> "
           "get_all_targets(200), tree queue, targets all-gathered" % (per_gpu, iters)}[config],
        "per_gpu": per_gpu,
        # a continuous loop where the workload is one (config 3: consecutive batches on streams; config 5:
        # data rounds through one tree queue), value_one_batch the median of one batch / round alone
        "value": streams["value"] if streams else rounds["value"] if rounds else med["value"],
        "unit": "trees/s" if config == 5 else "decisions/s",
        "value_one_batch": med["value"], "streams": streams, "rounds": rounds,
        "carry_out_per_s": med["carry_out_per_s"], "reps": len(reps), "median": med,
        "all_reps_value": [r["value"] for r in reps],
        "roofline": roof}
    if cpu and world == 1 and not args.no_cpu_baseline:
        w = None
        if config == 4:
            from citadels_self_play_amd import models
            w = [t.numpy() for t in models.fold(_cpu_model())]
        nc, ec = pool_caps(iters) if config == 5 else (node_cap, 5 * node_cap)
        try:
            out["cpu_baseline"] = cfr_cpu_baseline(config, iters, args.cfr_cpu_seconds, nc, ec, w)
        except Exception as e:
            out["cpu_baseline"] = {"error": str(e)[:300]}
    return out


def _cfr_streams(args, world, rank, dev, iters, per_gpu, node_cap):
    """Config 3 as a continuous self-play loop: K consecutive batches of
    `per_gpu` positions (built untimed) whose searches are launched
    round-robin on S HIP streams, so the next batch's trees take the SIMD
    slots the finished trees of earlier batches free (a launch lasts as long
    as its longest tree).  Decisions of all ranks / max-over-ranks time."""
    from citadels_self_play_amd import selfplay
    from citadels_self_play_amd.engine import ERR_OVERFLOW, GameBatch, side_streams
    K, S = args.cfr_stream_batches, args.cfr_streams
    batches = []
    for k in range(K + S):
        seeds = selfplay.shard(per_gpu * world, base_seed=CFR_SEED + 50_000_000 + k * 1_000_000)
        b = GameBatch(seeds, preset=True, device=dev)
        b.advance_random(0, 300)
        b.seed_numpy()
        b._pool(node_cap, 5 * node_cap)
        batches.append(b)
    torch.cuda.synchronize()
    sts = side_streams(dev, S)
    for i, st in enumerate(sts):                       # warm each stream's queue (untimed batches)
        with torch.cuda.stream(st):
            batches[K + i]._cfr_decide(iters, node_cap, 5 * node_cap)
    torch.cuda.synchronize()
    out = []
    _barrier(world)
    t0 = time.perf_counter()
    for k, b in enumerate(batches[:K]):
        with torch.cuda.stream(sts[k % S]):
            out.append(b._cfr_decide(iters, node_cap, 5 * node_cap)[1])
    torch.cuda.synchronize()
    _barrier(world)
    el = time.perf_counter() - t0
    st = torch.cat(out).to(torch.float64)
    over = int(((torch.cat(out)[:, 4] & ERR_OVERFLOW) != 0).sum())
    el, units, carry, over = _reduce([el, st.shape[0], st[:, 3].sum(), over], world, dev, maxes=(0,))
    return {"value": units / el, "carry_out_per_s": carry / el, "batches": K, "streams": S, "seconds": el,
            "overflow_lanes": int(over),
            "note": "K batches of positions searched round-robin on S HIP streams (untimed position setup); "
                    "value_one_batch is the median of one batch at a time"}


def _cfg5_rounds(args, world, rank, dev, iters, per_gpu):
    """Config 5 as train_from_scratch generates it: train_from_scratch.collect
    itself (its cross-round tree queue with the lookahead's admission rule --
    round r + 1 enters once round r's first walked trees project a shortfall
    -- and the async target all-gathers that keep a rank's slices running
    while it waits for slower ranks) for `--cfg5-rounds` data rounds of
    `per_gpu` trees per GPU (min_targets unbounded, so every round is needed
    and no round past the last is started).  `value` = all trees / the whole
    run, the first round's ramp and the last round's tail included."""
    from types import SimpleNamespace
    from citadels_self_play_amd import train_from_scratch as tfs
    # the same trees whatever the round size (5@960 runs twice the rounds of 1,920-tree ones), so the
    # first round's ramp and the last round's tail weigh the same in every leg
    R = max(args.cfg5_rounds, -(-args.cfg5_rounds * args.cfg5_trees // per_gpu))
    targs = SimpleNamespace(iters=iters, games_per_gpu=per_gpu, node_cap=None, seed=CFR_SEED + 90_000_000,
                            on_error="drop", save_tuples=False, lookahead=True)
    # the queue's node arena (~230 GB) is allocated before the timed region, as the one-round reps' warm-up
    # allocates theirs: a fresh hipMalloc of it after earlier legs released theirs takes ~6 s
    # (profiles/r06/cfg5_alloc), which a training run pays once per process -- its later rounds and phases
    # reuse the cached arena (engine.device_avail_bytes counts it as free, so the same size is asked for)
    t_alloc = time.perf_counter()
    warm = tfs._Lookahead(targs, world, 0, 10 ** 15, lambda m: None, R)
    warm.q.add(tfs.round_seeds(targs, world, 0, 0))
    warm.close()
    warm = None
    torch.cuda.synchronize()
    t_alloc = time.perf_counter() - t_alloc
    _barrier(world)
    t0 = time.perf_counter()
    log = (lambda m: print("cfg5 rounds %7.2f s: %s" % (time.perf_counter() - t0, m), file=sys.stderr, flush=True)) \
        if rank == 0 else (lambda m: None)
    feat, value, _ = tfs.collect(rank, world, targs, 0, 10 ** 15, log, max_rounds=R)
    torch.cuda.synchronize()
    _barrier(world)
    el = time.perf_counter() - t0
    done = [t - t0 for t in tfs.collect.round_done]
    dropped = sum(tfs.collect.dropped.values())
    el, trees, dropped, *done = _reduce([el, per_gpu * world * R, dropped] + done, world, dev,
                                        maxes=(0,) + tuple(range(3, 3 + R)))
    gaps = [b - a for a, b in zip(done, done[1:])]
    return {"value": trees / el, "unit": "trees/s", "rounds": R, "trees_per_round": per_gpu * world,
            "seconds": el, "round_done_s": done, "first_round_s": done[0],
            "later_round_s": sum(gaps) / len(gaps) if gaps else None, "arena_alloc_s_untimed": t_alloc,
            "dropped_trees": int(dropped), "pooled_targets": int(feat.shape[0]), "queue_rank0": tfs.collect.queue,
            "loop": "train_from_scratch.collect (lookahead admission, async all-gathers)",
            "note": "value = all rounds' trees / the whole run; one round alone is value_one_batch"}


def _mlp_rows(dev, rows):
    """encode_game rows of `rows` config-4 positions (the rows cfr_pred's rounds
    mode hands the value net: one leaf per suspended tree)."""
    from citadels_self_play_amd import _lib, selfplay
    from citadels_self_play_amd.engine import GameBatch
    b = GameBatch(selfplay.shard(rows, base_seed=CFR_SEED + 7_000_000), preset=True, device=dev)
    b.advance_random(0, 300)
    feat = torch.zeros((rows, 418), dtype=torch.float32, device=dev)
    _lib.check(b.lib.cit_encode_games(b.games.data_ptr(), rows, -1, feat.data_ptr(),
                                      torch.cuda.current_stream(dev).cuda_stream), "cit_encode_games")
    return feat


def run_mlp(dev, calls=20, warm=3, rows=MLP_ROWS, trace=None):
    """The value net's MFMA forward (ValueNet.forward: k_mlp_layer x 2 +
    k_mlp_head, v_mfma_f32_16x16x4_f32) on `rows` encode_game rows, as
    cfr_pred's rounds mode calls it: HIP events around each call on the
    stream it runs on; TF/s = MLP_FLOP_PER_ROW x rows / time against the fp32
    matrix peak.  `trace`: the kernel trace's per-call kernel time (summed
    durations of the three kernels, launch gaps excluded)."""
    net = _value_net(dev)
    feat = _mlp_rows(dev, rows)
    for _ in range(warm):
        net.forward(feat)
    st = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
    torch.cuda.synchronize()
    for a, b in evs:
        a.record(st)
        net.forward(feat)
        b.record(st)
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
    flop = MLP_FLOP_PER_ROW * rows
    out = {"kernel": "+".join(MLP_KERNELS) + " (ValueNet.forward, fp32 MFMA 16x16x4)", "rows": rows,
           "flop_per_row": MLP_FLOP_PER_ROW, "call_ms_events": ms, "calls": calls,
           "tflops_events": flop / (ms * 1e-3) / 1e12, "peak": FP32_MATRIX_PEAK_TF, "unit": "TFLOP/s",
           "path": "cfr_pred rounds mode's leaf batch (engine.GameBatch._cfr_pred: one row per suspended tree); "
                   "config 4's timed path evaluates leaves inside the search kernel instead (cit_mlp_wave.h)"}
    km = (trace or {}).get("kernel_ms_per_call")
    out["kernel_ms"] = km if km else ms
    out["kernel_ms_source"] = ("rocprofv3 --kernel-trace (summed kernel durations per call, in-run child)" if km
                               else "HIP events around each call")
    out["tflops"] = flop / (out["kernel_ms"] * 1e-3) / 1e12
    out["frac"] = out["tflops"] / FP32_MATRIX_PEAK_TF
    if trace:
        out["trace"] = trace
    return out


def _cpu_model():
    from citadels_self_play_amd import models
    torch.manual_seed(0)
    return models.ValueOnlyNN(418, 512).eval()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5),
                    help="headline workload (BASELINE configs; 2 = the metric's own)")
    ap.add_argument("--batch", type=int, default=4096, help="games per batch per GPU (config 2)")
    ap.add_argument("--games-per-block", type=int, default=0, help="0 = k_rollout_u (one game per workgroup)")
    ap.add_argument("--streams", type=int, default=3,
                    help="HIP streams the K timed batches are launched round-robin on (1 = one after another)")
    ap.add_argument("--queue", action="store_true",
                    help="config 2: the K timed batches as one work queue (cit_rollout_queue) instead of streams")
    ap.add_argument("--cpu-seconds", type=float, default=5.0, help="per C++ CPU-baseline leg")
    ap.add_argument("--py-seconds", type=float, default=2.0, help="Python-oracle CPU figure")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the in-run rocprofv3 --pmc passes")
    ap.add_argument("--no-cfr", action="store_true", help="skip the configs 3-5 legs (cfr_configs)")
    ap.add_argument("--cfr-configs", default="3,4,5,4@512,5@960",
                    help="configs 3-5; C@N runs config C at N positions / trees per GPU (4@512: the per-rank shard of "
                         "config 4's 4096 positions over 8 GPUs; 5@960: train_from_scratch's --games-per-gpu)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cfr-reps", type=int, default=5, help="timed reps of configs 3 and 4 (median reported)")
    ap.add_argument("--cfg5-reps", type=int, default=1, help="timed reps of config 5")
    ap.add_argument("--cfr-cpu-seconds", type=float, default=4.0, help="per C++ CPU-baseline leg of configs 3-5")
    ap.add_argument("--cfr-streams", type=int, default=3,
                    help="config 3: HIP streams for consecutive batches (3: 169-172 k vs 2: 124 k vs 4: 120-122 k, 'profiles/r05/config3_streams')")
    ap.add_argument("--cfr-stream-batches", type=int, default=12, help="config 3: batches in the streams run")
    ap.add_argument("--cfg5-trees", type=int, default=1920, help="config 5 trees per GPU")
    ap.add_argument("--cfg5-iters", type=int, default=200000, help="config 5 cfr_train iterations per tree")
    ap.add_argument("--cfg5-rounds", type=int, default=3,
                    help="config 5: data rounds through one cross-round tree queue (the `rounds` figure; 1 = off)")
    ap.add_argument("--no-mlp", action="store_true", help="skip the value-net MFMA figure (`mlp`)")
    ap.add_argument("--full-out", default="gpurun_out/bench/bench_full.json",
                    help="the full bench object (the stdout line is its compact summary)")
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
    cfr_list = [] if args.no_cfr or args.config != 2 else [c.strip() for c in args.cfr_configs.split(",") if c.strip()]

    if args.pmc_child:          # the counter runs of pmc_in_run_cfr: configs 3, 4, 5 once each, small
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        args.cfr_streams = 1
        line = {"pmc_child": 1}
        from citadels_self_play_amd import engine
        for key, c, n in PMC_CHILD_LEGS:
            import gc                  # as the main run: each leg from an empty allocator cache, so a leg's
            gc.collect()               # trees take the same path (tree queue or one launch) as its timed run
            torch.cuda.empty_cache()
            before = dict(engine.LAUNCHES)
            r = run_cfr(c, args, 1, 0, dev, cpu=False, per_gpu=n, warm_rep=False, n_reps=1)
            m = r["median"]
            line[key] = {"carry_outs": m["carry_out_per_s"] * m["seconds"], "search_ms": m["seconds"] * 1e3,
                         "launches": {k: engine.LAUNCHES.get(k, 0) - before.get(k, 0) for k in SEARCH_KERNELS
                                      if engine.LAUNCHES.get(k, 0) - before.get(k, 0)}}
        if not args.no_mlp:
            m = run_mlp(dev, calls=10, warm=2)
            line["mlp"] = {"calls": 12, "rows": m["rows"]}
        print(json.dumps(line), flush=True)
        return

    # The PMC passes run as child processes before this process touches the GPU.
    pmc = pmc_in_run(2) if (args.config == 2 and world == 1 and not args.no_pmc) else None
    if pmc is not None:
        pmc["trace"] = trace_in_run(args)
    cfr_pmc = pmc_in_run_cfr() if (world == 1 and not args.no_pmc and (cfr_list or args.config != 2)) else {}
    cfr_trace = trace_in_run_cfr() if (world == 1 and not args.no_pmc and (cfr_list or args.config != 2)) else {}

    dev = torch.device("cuda", local % max(1, n_dev))
    if world > 1:
        torch.cuda.set_device(dev)
        dist.init_process_group(args.dist_backend)
    torch.cuda.set_device(dev)

    if args.config == 2:
        out = run_rollout(args, world, rank, dev, n_dev, pmc)
        if rank == 0:
            _progress("config 2 done: %.4g carry_out/s" % out["value"])
    else:
        c = run_cfr(args.config, args, world, rank, dev, pmc=cfr_pmc.get(str(args.config)),
                    trace=cfr_trace.get(str(args.config)))
        out = None
        if rank == 0:
            out = {"metric": "MCCFR config %d" % args.config, "value": c["value"], "unit": c["unit"],
                   "n_gpus": min(world, max(1, n_dev)), "steps": c["reps"], "warmup": 1,
                   "ms_per_step": c["median"]["seconds"] * 1e3, "higher_is_better": True, "scaling": "weak",
                   "vs_baseline": None, "dtype": "f64", "data": "synthetic seeded positions",
                   "config": {"workload": c["workload"], "parallelism": "dp%d" % world},
                   "roofline": c["roofline"], "cpu_baseline": c.get("cpu_baseline"), "cfr": c}
    cfr_out = {}
    for key in cfr_list:
        # each leg starts from an empty allocator cache (outside every timed region): the legs' node
        # pools differ in size, and one leg's cached arena must not crowd the next leg's
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        try:
            c, _, n = key.partition("@")
            c = int(c)
            r = run_cfr(c, args, world, rank, dev, pmc=cfr_pmc.get(key), per_gpu=int(n) if n else None,
                        cpu=not n, trace=cfr_trace.get(key))
            if n and r is not None:
                r["shard_of"] = {4: "config 4's 4096 positions over 8 GPUs (the per-rank work of that config)",
                                 5: "config 5 / train_from_scratch at half its default --games-per-gpu"}.get(c)
            cfr_out[key] = r
            if rank == 0:
                _progress("cfr leg %s done: %.4g %s" % (key, r["value"], r["unit"]))
        except Exception as e:          # a CFR leg must not cost the headline line
            cfr_out[key] = {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}
    if cfr_pmc.get("error") and rank == 0:
        cfr_out["pmc_error"] = cfr_pmc["error"]
    if cfr_trace.get("error") and rank == 0:
        cfr_out["trace_error"] = cfr_trace["error"]
    mlp = None
    if args.config == 2 and not args.no_mlp and cfr_list:
        try:
            mlp = run_mlp(dev, trace=cfr_trace.get("mlp"))
        except Exception as e:          # nor the value-net figure
            mlp = {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}

    if rank == 0:
        if folded:
            out["folded"] = True
            out["ranks"] = world
        if args.config == 2:
            if world == 1 and not args.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.py_seconds)
            else:
                out["cpu_baseline"] = None
        if cfr_list:
            out["cfr_configs"] = cfr_out
        if mlp is not None:
            out["mlp"] = mlp
        if cfr_trace:
            out["cfr_trace"] = cfr_trace
        # the full object (counter passes, traces, notes) goes to a file beside the profiler CSVs; stdout
        # gets one compact line (< LINE_MAX_BYTES) naming it
        full = os.path.join(ROOT, args.full_out) if not os.path.isabs(args.full_out) else args.full_out
        detail = os.path.relpath(full, ROOT) if full.startswith(ROOT) else full
        try:
            os.makedirs(os.path.dirname(full), exist_ok=True)
            for src, name in (((pmc or {}).get("trace") or {}).get("stats_csv"), "rollout_kernel_stats.csv"), (
                    cfr_trace.get("_stats_csv"), "cfr_kernel_stats.csv"):
                if src and os.path.exists(src):
                    shutil.copy(src, os.path.join(os.path.dirname(full), name))
            with open(full, "w") as f:
                json.dump(out, f, indent=1)
        except OSError as e:
            detail = "not written: %s" % e
        line = compact_line(out, detail)
        txt = json.dumps(line)
        if len(txt) > LINE_MAX_BYTES:        # never again an unparseable line: drop the CFR legs' detail first
            line["cfr_configs"] = {k: _pick(v, "value", "value_one_batch", "unit") if isinstance(v, dict) else v
                                   for k, v in (line.get("cfr_configs") or {}).items()}
            txt = json.dumps(line)
        print(txt, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
