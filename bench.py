"""Benchmark: Option.carry_out transitions/s, batched 6-player self-play.

Workload (BASELINE.json configs[1], "config 2"): per GPU, 4096 preset
6-player games (run_utils.create_game) played by the uniform random policy
to terminal.  One bench step = one launch of the fused rollout kernel over a
fresh batch of 4096 games already resident in HBM (initialised, untimed,
before the timed region); seeds are disjoint across steps and ranks
(seed = base + (step * world + rank) * B + lane), so N GPUs play N x 4096
independent games per step (weak scaling, no data-path collective).

Prints ONE JSON line on rank 0.  `value` = carry_out transitions of all ranks
/ max-over-ranks wall time of the K timed steps.  `roofline` prices the
rollout kernel by its algorithmic bytes (2 x CIT_GAME_BYTES per transition,
SURVEY §8(d)) over its HIP-event duration; `cpu_baseline` times the CPU
oracle (oracle/citadels_oracle.py) on a bounded sample on rank 0 at N=1.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BASE_SEED = 1_000_000_000


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


def cpu_baseline(procs, budget_s):
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        res = pool.map(_oracle_worker, [(BASE_SEED + 10**8 + i * 10**6, budget_s) for i in range(procs)])
    wall = time.perf_counter() - t0
    steps = sum(r[0] for r in res)
    games = sum(r[1] for r in res)
    busy = max(r[2] for r in res)
    return {"value": steps / busy, "unit": "carry_out transitions/s", "cores": procs, "kind": "port",
            "sample": "%d preset games, uniform random policy to terminal, CPU oracle (pure Python), "
                      "%d processes x %.0f s (%.1f s wall incl. startup)" % (games, procs, budget_s, wall)}


def pmc_traffic():
    """HBM bytes per rollout launch from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_rollout_latest.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="games per GPU")
    ap.add_argument("--games-per-block", type=int, default=0, help="0 = auto (1 game per wavefront at B=4096)")
    ap.add_argument("--cpu-procs", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, the real path); gloo only to rehearse N>1 ranks on one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; modulo only matters when rehearsing N ranks on fewer GPUs
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    if world > 1:
        torch.cuda.set_device(dev)
        dist.init_process_group(args.dist_backend)
    torch.cuda.set_device(dev)

    from citadels_self_play_amd import layout as L
    from citadels_self_play_amd.engine import GameBatch

    B, K, W = args.batch, args.steps, args.warmup
    seer = None
    batches = []
    for step in range(W + K):
        s0 = BASE_SEED + (step * world + rank) * B
        gb = GameBatch(np.arange(s0, s0 + B), preset=True, device=dev, games_per_block=args.games_per_block,
                       seer=seer)
        seer = gb.seer
        batches.append(gb)
    torch.cuda.synchronize()

    for gb in batches[:W]:
        gb.rollout()
    torch.cuda.synchronize()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, gb in enumerate(batches[W:]):
        evs[k][0].record()
        gb.rollout()
        evs[k][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    trans_rank = sum(int(gb.steps.sum().item()) for gb in batches[W:])
    errs = sum(int((gb.errors() != 0).sum().item()) for gb in batches[W:])
    unfinished = sum(int((~gb.terminal()).sum().item()) for gb in batches[W:])
    t = torch.tensor([elapsed, float(trans_rank), float(errs), float(unfinished)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
    trans_all, errs_all, unfinished_all = float(t[1]), int(t[2]), int(t[3])

    if rank == 0:
        per_launch_trans = trans_rank / K
        avg_ms = float(np.mean(kernel_ms))
        alg_bytes = per_launch_trans * 2 * L.GAME_BYTES
        achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
        traffic = pmc_traffic()
        out = {
            "metric": "Option.carry_out steps/sec (whole node), 6-player batched self-play",
            "value": trans_all / elapsed,
            "unit": "carry_out transitions/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: seeded preset games (run_utils.create_game), CPython-MT19937 random policy, "
                    "bit-exact with the reference per seed",
            "config": {"workload": "config2: %d preset 6-player games per GPU, uniform random policy to terminal"
                                   % B, "games_per_gpu": B, "games_per_block": args.games_per_block,
                       "rng": "per-game CPython MT19937 (parity mode)", "parallelism": "dp%d" % world},
            "transitions_per_step": trans_all / K,
            "lane_errors": errs_all,
            "unfinished_lanes": unfinished_all,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_rollout", "kernel_avg_ms": avg_ms,
                         "alg_bytes_per_launch": alg_bytes,
                         "alg_bytes_per_transition": 2 * L.GAME_BYTES},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_procs, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
