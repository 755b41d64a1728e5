#!/usr/bin/env python3
"""Benchmark: batched state-based CRDT merge on MI355X.

Headline (BASELINE.json `metric`): merged Orswot objects/s on config 3 —
1M objects x ~32 members x 16 actors incl. deferred removes — plus the
achieved HBM GB/s of the merge kernel against the MI355X roofline.

A step = one pass of the hot path over one batch: out[i] = L[i].merge(&R[i])
for every object of the GPU's shard (one kernel launch), inputs resident in
HBM. Objects shard across ranks (weak scaling: 1M objects per GPU, object i
generated from SplitMix64(seed ^ i) so the data is identical at any N); there
is no collective on this path.

    python bench.py [--gpus N --steps K --warmup W] [--workload orswot|gcounter|pncounter|...]
    torchrun --nproc-per-node N bench.py --gpus N ...

Before the W untimed warmup steps, the step itself runs untimed and back to
back for --settle-ms (default 200 ms, the same count on every rank): the
part's clock settles over ~25 ms of continuous launches after the inputs are
generated, so with a small W the timed steps would otherwise measure the ramp
(DESIGN.md §9). The line reports it under `settle`.

At N > 1 without a launcher (no WORLD_SIZE in the environment) this process
starts N worker processes of itself (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_* set, one GPU each) before it makes any GPU call, relays rank 0's
line and exits with the workers' status. At N > 1 the headline line also
carries `anti_entropy`: configs 4 and 5 (BASELINE.json configs[3], [4]) over
RCCL, each checked after its timed steps (identical digests on every rank,
and a sample equal to a locally computed rank-order fold).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))

HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md: 8.0 TB/s spec
TRAFFIC_ROUNDS = ("r06", "r05", "r04", "r03q", "r03p", "r03n", "r03k", "r03j", "r03", "r02", "r01e")  # profiles/traffic_<round>[_<workload>].json, newest first
METRIC = "merged objects/sec (node) + achieved HBM GB/s % of peak, Orswot 1M×32 members"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 100 timed steps: the timed region's fixed ends (the first launch's
    # submission, the final synchronisation: ~0.1-0.2 ms) spread over 75 ms
    p.add_argument("--steps", type=int, default=100)
    # 50 untimed steps: the part's clock settles over the first ~30 back-to-back
    # launches after the inputs are generated (tools/steady_probe.py: 0.88 ->
    # 0.75 ms per headline launch); the timed steps then see the steady state
    p.add_argument("--warmup", type=int, default=50)
    # before the W warmup steps, untimed launches of the same step until the
    # device has run it for this long: the clock ramp is a matter of time
    # (~25 ms of back-to-back launches), not of step count, so a small W
    # (the driver's 5 x 0.75 ms) would otherwise time the ramp
    p.add_argument("--settle-ms", type=float, default=200.0)
    p.add_argument("--workload", default="orswot",
                   choices=["orswot", "orswot_tail", "orswot_csr_tail", "vclock", "gcounter", "pncounter", "orswot_csr", "gcounter_ae", "bincode", "apply",
                            "mvreg", "map", "map_orswot", "map_map", "clock_csr", "truncate", "spawn_check"])
    p.add_argument("--replicas", type=int, default=8, help="orswot_csr at N=1: replicas folded locally")
    p.add_argument("--n-actors", type=int, default=16,
                   help="orswot: dense top-clock actors (config 3: 16; 33-64 take the 64-bit actor-mask join, "
                        "65-1024 the dense-wide mask join over each object's present actors)")
    p.add_argument("--gen-params", default=None,
                   help="orswot: JSON overrides of the op-simulation generator's parameters (crdt_orswot_gen_params), "
                        "e.g. the wide-union distribution of DESIGN.md §11")
    p.add_argument("--n-obj", type=int, default=None, help="objects per GPU")
    p.add_argument("--threads", type=int, default=16, help="host threads for input generation")
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="CPU-baseline threads (default: every host core, os.cpu_count() = nproc)")
    p.add_argument("--cpu-sample", type=int, default=500_000, help="objects in the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-anti-entropy", action="store_true",
                   help="N > 1: skip the config-4/5 anti-entropy sub-measurements of the headline line")
    p.add_argument("--ae-steps", type=int, default=3, help="timed steps of each anti-entropy sub-measurement")
    p.add_argument("--ae-deadline", type=float, default=300.0,
                   help="N > 1: seconds the anti-entropy sub-measurements may take; past it every rank ends the run "
                        "and rank 0 prints the headline line with the anti-entropy part marked unfinished")
    p.add_argument("--ae-n-obj", type=int, default=None,
                   help="objects of the anti-entropy sub-measurements (default: the configs' own sizes)")
    p.add_argument("--rehearse", action="store_true",
                   help="rehearse the N > 1 logic on ONE GPU: every rank on cuda:0, gloo collectives, the Orswot "
                        "join through crdt_orswot_replica_join_transport (tests; not a measurement)")
    p.add_argument("--traffic-json", default=next(
        (f for f in (os.path.join(REPO, "profiles", f"traffic_{r}.json") for r in TRAFFIC_ROUNDS) if os.path.exists(f)),
        None),
                   help="measured per-launch HBM bytes (rocprofv3 PMC) to report as roofline.traffic")
    return p.parse_args()


def spawn_ranks(args):
    """--gpus N > 1 without a launcher: start N fresh worker processes of this
    script, one per GPU (RANK = LOCAL_RANK = r), rendezvous on 127.0.0.1. This
    process never touches the GPU (no torch import before or after). Rank 0
    prints the JSON line; the exit code is the first failing worker's (the
    others are stopped then, so none waits in a collective forever)."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the others", file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc if rc >= 0 else 128 - rc


def dist_setup(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.workload == "spawn_check":  # CPU only: the launch path itself (tests/test_bench_spawn.py)
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
        return rank, world, local
    if args.rehearse:  # every rank on the one GPU, gloo: no RCCL (it cannot put two ranks on one GPU)
        local = 0
        torch.cuda.set_device(0)
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
        return rank, world, local
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device(f"cuda:{local}"))
    return rank, world, local


def barrier(world):
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    import torch
    import torch.distributed as dist

    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world):
    import torch
    import torch.distributed as dist

    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def load_traffic(path, key):
    try:
        with open(path) as f:
            return json.load(f).get(key)
    except (OSError, ValueError, TypeError):
        return None


def wl_traffic(args, workload, *kernels):
    """Per-launch HBM bytes of the workload's measured kernels from its
    rocprofv3 FETCH_SIZE/WRITE_SIZE passes (tools/profile_workload.sh +
    tools/traffic.py -> profiles/traffic_<round>_<workload>.json, newest round first),
    summed over the kernels one measured launch runs (every instantiation of a
    templated one: tools/traffic.py keys them <kernel>_<last template argument>);
    None off the profiled (default) size."""
    if args.n_obj is not None:
        return None
    path = None
    for rnd in TRAFFIC_ROUNDS:
        path = os.path.join(REPO, "profiles", f"traffic_{rnd}_{workload}.json")
        if os.path.exists(path):
            break
    try:
        with open(path) as f:
            tab = json.load(f)
    except (OSError, ValueError, TypeError):
        return None
    vals = []
    for k in kernels:
        hits = [v for n, v in tab.items() if n != "detail" and (n == k or n.startswith(k + "_"))]
        vals.append(sum(hits) if hits else None)
    return None if any(v is None for v in vals) else float(sum(vals))


def cpu_quota():
    """CPUs this process may actually use: the affinity set, capped by the
    cgroup CPU quota (cpu.max / cfs_quota_us) where one is set — on the GPU box
    nproc shows the whole machine while the job's quota is a share of it."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for path, two in (("/sys/fs/cgroup/cpu.max", True), ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", False)):
        try:
            txt = open(path).read().split()
            if two:
                q, per = txt[0], txt[1]
            else:
                q, per = txt[0], open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().split()[0]
            if q not in ("max", "-1"):
                n = min(n, max(1, -(-int(q) // int(per))))
            break
        except (OSError, IndexError, ValueError):
            continue
    return n


def cpu_threads(args):
    """CPU-baseline threads: one per host core this job can use (BASELINE.md's
    "one std::thread per host core", standing in for rayon over objects).
    That is nproc unless a cgroup quota caps the job below it; both are reported."""
    return max(1, args.cpu_threads or cpu_quota())


def cpu_cores_note():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_quota": cpu_quota()}


def gen_params(args, A):
    """The orswot generator's parameters: config 3's, with --n-actors and
    --gen-params (JSON) applied; None for config 3 itself."""
    if A == 16 and not args.gen_params:
        return None
    p = {"n_actors": A}
    if args.gen_params:
        p.update(json.loads(args.gen_params))
    return p


def run_orswot(args, rank, world, local):
    import numpy as np
    import torch

    import crdts_hip

    n = args.n_obj or 1_000_000
    first = rank * n
    t0 = time.time()
    A = args.n_actors
    tail = args.workload in ("orswot_tail", "orswot_csr_tail")
    csr = args.workload == "orswot_csr_tail"
    flags = crdts_hip.SPARSE_CLOCK if csr else 0
    if csr:  # config 5's CSR records (replicas 0 and 1) with the same heavy tail
        A = crdts_hip.CONFIG5["universe"]
        (lb, lo), (rb, ro) = crdts_hip.generate_orswot_csr_tail(n, first_obj=first, threads=args.threads)
    elif tail:  # config 3 with a heavy tail: 5 % of the objects at 100 / 300 / 1000 members per side
        A = 16
        (lb, lo), (rb, ro) = crdts_hip.generate_orswot_tail(n, first_obj=first, threads=args.threads)
    else:
        (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, first_obj=first, threads=args.threads,
                                                       params=gen_params(args, A))
    gen_s = time.time() - t0
    eng = crdts_hip.Engine(local)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, A, device=local, flags=flags)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, A, device=local, flags=flags)
    out = eng.orswot_alloc_out(L, R)
    stream = torch.cuda.Stream(device=local)
    # one checked launch, then algorithmic bytes from the real output sizes
    eng.orswot_merge(L, R, out=out, stream=stream, check_status=True)
    out_sizes = out.base.view(torch.int32)[(out.off // 4)].cpu().numpy().astype(np.int64)
    in_bytes = int(lb.nbytes + rb.nbytes)
    out_bytes = int(out_sizes.sum())
    rec_bytes = in_bytes + out_bytes + 3 * 8 * n  # record bytes: + L/R offsets read, out offsets written
    # the roofline numerator: SURVEY.md §8(d)'s compact bytes of both inputs
    # and the output (no headers, padding or offsets), from the records' headers
    alg_bytes = L.compact_bytes() + R.compact_bytes() + out.compact_bytes()

    settle(args, stream, lambda: eng.orswot_merge(L, R, out=out, stream=stream, check_status=False), world)
    for _ in range(args.warmup):
        eng.orswot_merge(L, R, out=out, stream=stream, check_status=False)
    ev = TimingEvents(args.steps)  # HIP events around every launch (timing only: no system fence)
    barrier(world)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev.record(k, False, stream)
        eng.orswot_merge(L, R, out=out, stream=stream, check_status=False)
        ev.record(k, True, stream)
    stream.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    eng.status(stream)  # no record-level errors latched during the timed steps
    kernel_ms = ev.mean_ms()
    wall = max_over_ranks(wall, world)
    total_objs = sum_over_ranks(float(n * args.steps), world)
    value = total_objs / wall
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    achieved_rec = rec_bytes / (kernel_ms * 1e-3) / 1e9
    # measured HBM bytes of one launch (both kernels of the timed window), from
    # the FETCH_SIZE / WRITE_SIZE passes of tools/profile.sh -> tools/traffic.py
    tk = [load_traffic(args.traffic_json, k)
          for k in ("orswot_join_kernel", "orswot_merge_general_kernel", "orswot_big_kernel")]
    traffic = None if args.n_obj is not None or A != 16 or tail or tk[0] is None else tk[0] + sum(t or 0.0 for t in tk[1:])
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "objects/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": ("synthetic: op-simulated Orswot replica pairs (SplitMix64 seed 0xC0FFEE05 ^ object id)" if csr else
                 "synthetic: op-simulated Orswot pairs (SplitMix64 seed 0xC0FFEE03 ^ object id)"),
        "config": {
            "workload": (f"orswot_csr_tail: config 5's CSR records (replicas 0 and 1, 1024-actor universe) with a "
                         f"heavy tail, {n} objects/GPU, every 20th object at "
                         f"{'/'.join(map(str, crdts_hip.TAIL_SIZES))} members per side in turn (the sparse general / "
                         "big-object path), the rest config-5 pairs") if csr else
                        (f"orswot_tail: config 3 with a heavy tail, {n} objects/GPU, every 20th object at "
                         f"{'/'.join(map(str, crdts_hip.TAIL_SIZES))} members per side in turn (the general / big-object "
                         "path), the rest config-3 pairs") if tail else
                        ("orswot_merge config3 (BASELINE.json configs[2]): 1M objects/GPU x ~31 members/side "
                         "x 16 dense actors incl. deferred removes") if A == 16 else
                        (f"orswot_merge config3 shape over {A} dense actors ("
                         + ("64-bit actor-mask join" if A <= 64 else "sparse mask join over the present actors, DN form")
                         + "): "
                         f"{n} objects/GPU incl. deferred removes"
                         + (f", generator {json.loads(args.gen_params)}" if args.gen_params else "")),
            "n_obj_per_gpu": n,
            "n_actors": A,
            "alg_bytes_per_merge": alg_bytes / n,
            "record_bytes_per_merge": rec_bytes / n,
            "parallelism": f"objects sharded over {world} GPU(s), no collective",
            "gen_s": round(gen_s, 2),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": ("orswot_big_kernel<CSR> (+ orswot_sparse_mask_kernel, orswot_sparse_general_kernel in the "
                       "same window)" if csr else
                       "orswot_big_kernel (+ orswot_join5_kernel, orswot_merge_general_kernel in the same window)"
                       if tail else ("orswot_join5_kernel (+ orswot_merge_general_kernel, orswot_big_kernel in the "
                                     "same window)" if A <= 64 else
                                     "orswot_sparse_mask_kernel<DN> (the dense-wide join; + orswot_dense_wide_kernel, "
                                     "orswot_merge_general_kernel, orswot_big_kernel in the same window)")),
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "kernel_ms": kernel_ms,
            "alg_bytes_per_launch": alg_bytes,
            "alg_bytes_def": "SURVEY.md §8(d) compact bytes of self + other + out (no header / padding / offsets)",
            "traffic": traffic,
            "record_bytes": {"per_launch": rec_bytes, "achieved": achieved_rec, "frac": achieved_rec / HBM_PEAK_GBS,
                             "def": "the record layout's bytes: headers, padding, + 3 x 8 B offsets per object"},
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_orswot(lb, lo, rb, ro, args)
    if world > 1:
        from crdts_hip import replica

        del L, R, out, lb, lo, rb, ro
        torch.cuda.empty_cache()
        dog0 = _ae_watchdog(args, rank, res)  # (the communicator's setup is bounded too)
        comm_ok = True
        if not args.rehearse:
            try:
                replica.init_comm(eng)  # the context's RCCL communicator: its rank count is reported
                res["comm"] = {"rccl_ranks": eng.comm_count()}
            except Exception as e:  # noqa: BLE001 — reported; the headline stands, anti-entropy skipped
                res["comm"] = {"error": f"{type(e).__name__}: {e}"[:400]}
                comm_ok = False
        if comm_ok:
            dog0.cancel()
        if comm_ok and not args.no_anti_entropy:
            # configs 4 and 5 over the same ranks (the driver's multi-GPU run
            # measures and checks them with the headline), each with its own
            # timed region, checked after it. A watchdog bounds them: the
            # headline is measured already, and a collective that never
            # returns must not cost it (_ae_watchdog)
            sub = argparse.Namespace(**vars(args))
            sub.steps, sub.warmup, sub.n_obj, sub.no_cpu_baseline = args.ae_steps, 1, args.ae_n_obj, True
            res["anti_entropy"] = {}
            dog = _ae_watchdog(args, rank, res)
            errored = False
            try:
                for key, fn in (("config4_gcounter", run_gcounter_ae), ("config5_orswot_csr", run_orswot_csr)):
                    try:
                        r = fn(sub, rank, world, local, eng=eng)
                    except Exception as e:  # noqa: BLE001 — reported in the line; the headline stands
                        # (peers may be left in a collective: the watchdog stays
                        # armed so that every rank still ends by the deadline)
                        res["anti_entropy"][key] = {"error": f"{type(e).__name__}: {e}"[:400]}
                        errored = True
                        break
                    res["anti_entropy"][key] = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "steps",
                                                                  "config", "comm", "check") if k in r}
                    torch.cuda.empty_cache()
            finally:
                if not errored:
                    dog.cancel()
    return res


_PRINT_LOCK = None
AE_TIMEOUT_EXIT = 3  # exit code of every rank the anti-entropy watchdog ends


def _emit(res):
    """Rank 0's one JSON line, printed at most once (the main thread or the
    anti-entropy watchdog, whichever comes first)."""
    global _PRINT_LOCK
    import threading

    if _PRINT_LOCK is None:
        _PRINT_LOCK = threading.Lock()
    with _PRINT_LOCK:
        if getattr(_emit, "done", False):
            return False
        _emit.done = True
        print(json.dumps(res), flush=True)
        return True


def _ae_watchdog(args, rank, res):
    """Past --ae-deadline seconds in the anti-entropy part, every rank ends
    the process with exit code AE_TIMEOUT_EXIT (non-zero: a hung or failed
    collective must not look like a clean run to the launcher); rank 0 first
    prints the line — the headline was measured and checked before it — with
    the unfinished sub-measurements marked. os._exit, not exec: nothing
    replaces the process."""
    import threading

    def fire():
        if rank == 0:
            out = dict(res)
            out["anti_entropy"] = dict(res.get("anti_entropy", {}))
            out["anti_entropy"]["unfinished"] = f"stopped after {args.ae_deadline:.0f} s (--ae-deadline)"
            if SETTLE:
                out["settle"] = dict(SETTLE)
            _emit(out)
        sys.stderr.write(f"bench.py rank {rank}: anti-entropy past --ae-deadline, exiting\n")
        sys.stderr.flush()
        os._exit(AE_TIMEOUT_EXIT)

    t = threading.Timer(args.ae_deadline, fire)
    t.daemon = True
    t.start()
    return t


def cpu_baseline_orswot(lb, lo, rb, ro, args):
    """The oracle (C++ std::map/unordered_map restatement of Orswot::merge with
    the reference's clone pattern) on the host cores, bounded sample."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi

    m = min(args.cpu_sample, len(lo))
    end = int(lo[m]) if m < len(lo) else lb.nbytes
    endr = int(ro[m]) if m < len(ro) else rb.nbytes
    threads = cpu_threads(args)
    secs = oracle_ffi.orswot_bench(lb[:end], lo[:m], rb[:endr], ro[:m], threads)
    m1 = max(1, m // 10)
    secs1 = oracle_ffi.orswot_bench(lb, lo[:m1], rb, ro[:m1], 1)
    return {
        "value": m / secs,
        "unit": "objects/s",
        "cores": threads,
        "kind": "port", **cpu_cores_note(),
        "sample": f"first {m} objects of the same batch, merge loop only (decode untimed), "
                  f"{threads} std::threads static partition",
        "value_1core": m1 / secs1,
    }


def run_vclock(args, rank, world, local):
    """Config 1 (BASELINE.json configs[0]): 1M VClock pairwise merges, 16
    actors, each present with p = 0.75, counters U[1, 2^32) (a drawn 0 is an
    absent actor, the same state), SplitMix64 seed 0xC0FFEE01. BASELINE.md
    names it CPU plumbing: the line reports the reference-shaped CPU merge
    (VClock::merge over std::map, src/vclock.rs:131-137) at 1 core and at every
    host core, with the GPU's dense_max_kernel merge of the same rows beside it
    (a step = one launch over the 1M pairs, rows resident in HBM)."""
    import numpy as np
    import torch

    import crdts_hip

    n, A = args.n_obj or 1_000_000, 16
    first = rank * n
    a = crdts_hip.generate_dense(n, A, seed=0xC0FFEE01, first_obj=first, bits=32, pct_zero=25, threads=args.threads)
    b = crdts_hip.generate_dense(n, A, seed=0xC0FFEE01 ^ 0x5EED, first_obj=first, bits=32, pct_zero=25,
                                 threads=args.threads)
    dev = f"cuda:{local}"
    da = torch.from_numpy(a.view(np.int64)).to(dev)
    db = torch.from_numpy(b.view(np.int64)).to(dev)
    eng = crdts_hip.Engine(local)
    stream = torch.cuda.Stream(device=local)
    eng.dense_merge(da, db, A, "vclock", stream=stream)
    eng.status(stream)
    assert (da.cpu().numpy().view(np.uint64) == np.maximum(a, b)).all()  # spot parity (pointwise max)

    def step():  # after the first merge self == max: same bytes read and written, same work
        eng.dense_merge(da, db, A, "vclock", stream=stream)

    wall, ev_ms = _timed_steps(args, world, stream, step)
    alg = 24.0 * n * A
    ach = alg / (ev_ms * 1e-3) / 1e9
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "VClock pairwise merges/sec (node), 16 actors",
        "value": total / wall, "unit": "merges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic: SplitMix64 0xC0FFEE01, p(present)=0.75, counters U[1,2^32)",
        "config": {"workload": f"vclock config1 (BASELINE.json configs[0]): {n} VClock pairs x {A} actors",
                   "parallelism": f"dp{world} (pairs sharded)"},
        "roofline": {"bound": "hbm", "kernel": "dense_max_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms, "alg_bytes_per_launch": alg,
                     "traffic": None, "note": "128 MB per side: launch-latency-scale, not a roofline case"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_ffi

        th = cpu_threads(args)
        secs = oracle_ffi.dense_bench(a.ravel(), b.ravel(), A, th)
        m1 = n // 4
        secs1 = oracle_ffi.dense_bench(a[:m1].ravel(), b[:m1].ravel(), A, 1)
        res["cpu_baseline"] = {"value": n / secs, "unit": "merges/s", "cores": th, "kind": "port", **cpu_cores_note(),
                               "sample": f"all {n} pairs on {th} std::threads (+ {m1} pairs on 1 core), "
                                         "VClock::merge over std::map, conversion untimed",
                               "value_1core": m1 / secs1}
    return res


def run_dense(args, rank, world, local, kind):
    import numpy as np
    import torch

    import crdts_hip

    A = 64
    slots = A * (2 if kind == "pncounter" else 1)
    # configs[1]: 100M counters x 64 dense actors; PNCounter's [P|N] rows are
    # twice as wide, so it runs 50M rows per GPU to fit one HBM stack set.
    n = args.n_obj or (100_000_000 if kind == "gcounter" else 50_000_000)
    g = torch.Generator(device=f"cuda:{local}")
    g.manual_seed(0xC0FFEE02 + rank)
    a = torch.randint(0, 1 << 40, (n * slots,), dtype=torch.int64, device=f"cuda:{local}", generator=g)
    b = torch.randint(0, 1 << 40, (n * slots,), dtype=torch.int64, device=f"cuda:{local}", generator=g)
    a[torch.rand(n * slots, device=f"cuda:{local}", generator=g) < 0.25] = 0
    b[torch.rand(n * slots, device=f"cuda:{local}", generator=g) < 0.25] = 0
    eng = crdts_hip.Engine(local)
    stream = torch.cuda.Stream(device=local)
    torch.cuda.synchronize()  # generated on torch's stream; the merges run on `stream`
    settle(args, stream, lambda: eng.dense_merge(a, b, A, kind, stream=stream), world)
    for _ in range(args.warmup):
        eng.dense_merge(a, b, A, kind, stream=stream)
    ev = TimingEvents(args.steps)
    barrier(world)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev.record(k, False, stream)
        eng.dense_merge(a, b, A, kind, stream=stream)
        ev.record(k, True, stream)
    stream.synchronize()
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world)
    kernel_ms = ev.mean_ms()
    alg = 24.0 * n * slots
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": f"merged {kind} objects/sec (node), {A} dense actors",
        "value": total / wall, "unit": "objects/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic: U[0,2^40) with 25% zeros",
        "config": {"workload": f"{kind} dense merge (BASELINE.json configs[1])", "n_obj_per_gpu": n,
                   "n_actors": A, "parallelism": f"objects sharded over {world} GPU(s), no collective"},
        "roofline": {"bound": "hbm", "kernel": "dense_max_kernel", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "kernel_ms": kernel_ms,
                     "alg_bytes_per_launch": alg,
                     "traffic": wl_traffic(args, "gcounter", "dense_max_kernel") if kind == "gcounter" else None},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_ffi

        m = min(args.cpu_sample * 4, n)
        ha = a[: m * slots].cpu().numpy().view(np.uint64).copy()
        hb = b[: m * slots].cpu().numpy().view(np.uint64).copy()
        threads = cpu_threads(args)
        secs = oracle_ffi.dense_bench(ha, hb, slots, threads)
        res["cpu_baseline"] = {"value": m / secs, "unit": "objects/s", "cores": threads, "kind": "port", **cpu_cores_note(),
                               "sample": f"first {m} rows, VClock::merge over std::map, {threads} threads"}
    return res


class TimingEvents:
    """n (start, end) pairs of timing-only HIP events on torch's HIP runtime
    (the already-loaded libamdhip64, crdts_hip._lib.hip_runtime): created with
    hipEventDisableSystemFence, so recording one does not write back and
    invalidate the caches between two steps — a per-step torch event does,
    and that gap (~11 us per step, tools/steady_probe.py) is not part of the
    merge. Times are read after a stream synchronisation."""

    FLAGS = 0x20000000  # hipEventDisableSystemFence (hip_runtime_api.h)

    def __init__(self, n):
        import ctypes as C

        import torch  # noqa: F401  (its HIP runtime is the one bound below)

        from crdts_hip._lib import hip_runtime

        self.C = C
        self.hip = hip_runtime()
        self.hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
        self.hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        self.hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        self.hip.hipEventDestroy.argtypes = [C.c_void_p]
        self.ev = []
        for _ in range(2 * n):
            e = C.c_void_p()
            if self.hip.hipEventCreateWithFlags(C.byref(e), self.FLAGS) != 0:
                raise RuntimeError("hipEventCreateWithFlags failed")
            self.ev.append(e)

    def record(self, i, end, stream):
        if self.hip.hipEventRecord(self.ev[2 * i + int(end)], self.C.c_void_p(stream.cuda_stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def mean_ms(self):
        ms, out = self.C.c_float(), []
        for i in range(len(self.ev) // 2):
            if self.hip.hipEventElapsedTime(self.C.byref(ms), self.ev[2 * i], self.ev[2 * i + 1]) != 0:
                raise RuntimeError("hipEventElapsedTime failed")
            out.append(ms.value)
        return sum(out) / len(out)

    def __del__(self):
        for e in getattr(self, "ev", []):
            self.hip.hipEventDestroy(e)


SETTLE = {}  # the settle phase of this run, reported in the JSON line


def settle(args, stream, fn, world=1):
    """Untimed calls of fn() (the timed step itself), back to back, for about
    args.settle_ms of device time before the W warmup steps. The count comes
    from the slowest rank's time per call, so every rank makes the same number
    of calls (a step may hold collectives)."""
    if args.settle_ms <= 0:
        return
    # one probe call first: a step that alone outlasts the budget (the 64 GB
    # all-reduce of config 4 at N = 8) settles nothing more by repetition
    t0 = time.perf_counter()
    fn()
    stream.synchronize()
    per = max_over_ranks(time.perf_counter() - t0, world)
    probes = 1
    if 8.0 * per < args.settle_ms * 1e-3:  # short steps: the per-call time over 8 calls
        t1 = time.perf_counter()
        for _ in range(7):
            fn()
        stream.synchronize()
        per = max_over_ranks((time.perf_counter() - t1) / 7.0, world)
        probes = 8
    # the count from all-reduced values only: every rank makes the same number
    # of calls (a step may hold collectives; a locally measured elapsed time
    # would differ between ranks)
    n = min(4096, max(0, int(args.settle_ms * 1e-3 / max(per, 1e-6)) - probes))
    for k in range(n):
        fn()
        if k % 64 == 63:
            stream.synchronize()  # bounded queue depth
    stream.synchronize()
    SETTLE.update({"ms": round((time.perf_counter() - t0) * 1e3, 1), "launches": probes + n,
                   "note": "untimed calls of the timed step before the W warmup steps (the clock ramp, DESIGN.md §9)"})


def _timed_steps(args, world, stream, fn, on_settled=None):
    """settle + W warmup + K timed calls of fn(); returns (wall_s over ranks (max), mean event ms on `stream`).
    on_settled() runs between the settle phase and the warmup steps (counters
    per warmup + timed step start there)."""
    settle(args, stream, fn, world)
    if on_settled is not None:
        on_settled()
    for _ in range(args.warmup):
        fn()
    ev = TimingEvents(args.steps)
    barrier(world)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev.record(k, False, stream)
        fn()
        ev.record(k, True, stream)
    stream.synchronize()
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world)
    return wall, float(ev.mean_ms())


def _packed_digest(base_u8, used):
    """crdts_hip.replica.digest of a PACKED batch (records contiguous in object
    order from byte 0): sum over its u64 words w_k of w_k * (2k + 1) mod 2^64."""
    import numpy as np

    w = base_u8[:used].cpu().numpy().view(np.uint64)
    k = np.arange(w.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int((w * (k * np.uint64(2) + np.uint64(1))).sum(dtype=np.uint64))


def _gather_ints(vals, world):
    """All-gather a few u64 values (as int64 on the GPU) -> list per rank."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in vals], dtype=torch.int64, device="cuda")
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [[int(x) % (1 << 64) for x in p.cpu().tolist()] for p in parts]


def run_orswot_csr(args, rank, world, local, eng=None):
    """Config 5 (BASELINE.json configs[4]): 1M Orswots with CSR top clocks over
    a 1024-actor universe; replica anti-entropy. At N > 1 rank r holds replica
    r and a step is crdt_orswot_replica_join over RCCL (owner-sharded rank-order
    fold of the N replicas, into a reused output buffer); after the timed
    steps every rank's digest must be equal and a sample of objects from every
    range must equal the oracle's rank-order fold. At N = 1 a step folds
    `--replicas` replicas held locally (crdt_orswot_fold)."""
    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip import replica

    n = args.n_obj or 1_000_000
    R = world if world > 1 else args.replicas
    t0 = time.time()
    reps = crdts_hip.generate_replicas(n, R, threads=args.threads, keep=(rank, 1) if world > 1 else None)
    gen_s = time.time() - t0
    eng = eng or crdts_hip.Engine(local)
    SP, U = crdts_hip.SPARSE_CLOCK, crdts_hip.CONFIG5["universe"]
    stream = torch.cuda.Stream(device=local)
    check = None
    if world > 1:
        mine = crdts_hip.OrswotBatch.from_host(*reps[0], U, device=local, flags=SP)
        del reps
        if args.rehearse:  # the same C++ join over the gloo transport
            T = replica.GlooTransport()
            bound = int(sum_over_ranks(float((mine.bytes + 15) // 16 * 16), world))
            out = eng.orswot_replica_alloc_out(mine, bound)

            def step():
                return eng.orswot_replica_join_transport(mine, T, out=out, stream=stream)
        else:
            if not eng.has_comm:
                replica.init_comm(eng)  # the context's own RCCL communicator (crdt_comm_init)
            out = eng.orswot_replica_alloc_out(mine, eng.orswot_replica_join_bound(mine, stream))

            def step():  # owner-sharded: crdt_orswot_replica_join over RCCL, reused output
                return eng.orswot_replica_join(mine, out=out, stream=stream)
    else:
        batches = [crdts_hip.OrswotBatch.from_host(b, o, U, device=local, flags=SP) for b, o in reps]
        del reps
        # a step = crdt_orswot_fold (R - 1 batched merges, the intermediate
        # batches in the context's buffer, the output reused); the same fold
        # through explicit crdt_orswot_merge_ex calls into preallocated outputs
        # gives the intermediate records the algorithmic bytes count, and the
        # same final records (checked below)
        outs, acc = [], batches[0]
        for B in batches[1:]:
            outs.append(eng.orswot_alloc_out(acc, B))
            acc = outs[-1]

        def step_classic():
            acc = batches[0]
            for B, o in zip(batches[1:], outs):
                acc = eng.orswot_merge(acc, B, out=o, stream=stream, check_status=False)
            return acc

        fold_out = eng.orswot_fold(batches, stream=stream)

        def step():
            return eng.orswot_fold(batches, out=fold_out, stream=stream, check_status=False)

    final = step()
    eng.status(stream)
    syncs0 = {}
    wall, ev_ms = _timed_steps(args, world, stream, step, on_settled=lambda: syncs0.update(n=eng.host_syncs()))
    syncs_per_step = (eng.host_syncs() - syncs0["n"]) / float(args.warmup + args.steps)
    eng.status(stream)
    if world > 1:
        # self-check (outside the timed region): identical bytes on every rank,
        # and a sample of every rank's range equal to the oracle's fold
        final = step()
        torch.cuda.synchronize()
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_ffi

        dg = _packed_digest(final.base, final.bytes)
        digests = [g[0] for g in _gather_ints([dg], world)]
        b = replica.ranges(n, world)
        host_b = final.base[: final.bytes].cpu().numpy()
        host_o = final.off.cpu().numpy().view(np.uint64)
        bad, sampled = 0, 0
        for j in range(world):
            m = min(32, b[j + 1] - b[j])
            if m == 0:
                continue
            sub = crdts_hip.generate_replicas(m, R, first_obj=b[j], threads=4)
            acc = sub[0]
            for xb, xo in sub[1:]:
                acc = oracle_ffi.orswot_merge_batch(acc[0], acc[1], xb, xo, U, threads=4, flags=SP)
            for k in range(m):
                o = int(host_o[b[j] + k])
                size = int(host_b[o:o + 4].view(np.uint32)[0])
                eo = int(acc[1][k])
                esize = int(acc[0][eo:eo + 4].view(np.uint32)[0])
                bad += int(host_b[o:o + size].tobytes() != acc[0][eo:eo + esize].tobytes())
                sampled += 1
        check = {"digests_equal": len(set(digests)) == 1, "digest": f"{dg:016x}", "sample_objects": sampled,
                 "sample_mismatches": bad, "ok": len(set(digests)) == 1 and bad == 0}
        if not check["ok"]:
            print(f"bench.py rank {rank}: config-5 anti-entropy check FAILED: {check}", file=sys.stderr)
    merges = n * (R - 1)
    total = sum_over_ranks(float(merges * args.steps), world)
    res = {
        "metric": "replica anti-entropy: Orswot object merges/sec (node), CSR clocks, 1024-actor universe",
        "value": total / wall, "unit": "object-merges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: op-simulated replicas (SplitMix64 seed 0xC0FFEE05 ^ object id)",
        "config": {"workload": f"orswot_csr config5 (BASELINE.json configs[4]): {n} objects x {R} replicas, "
                               "CSR top clocks, fold ((r0 ⊔ r1) ⊔ r2) ...",
                   "replicas": R, "n_obj": n, "gen_s": round(gen_s, 2),
                   "parallelism": (("owner-sharded join over the gloo transport (crdt_orswot_replica_join_transport): "
                                    "slices of range j -> rank j, rank-order fold of n/N objects, folded ranges "
                                    "all-gathered") if args.rehearse else
                                   ("owner-sharded RCCL join: slices of range j -> rank j (send/recv), rank-order "
                                    "fold of n/N objects, folded ranges all-gathered (crdt_orswot_replica_join)"))
                   if world > 1 else "local fold"},
    }
    if world > 1:
        res["comm"] = {"rccl_ranks": None if args.rehearse else eng.comm_count(), "host_syncs_per_step": syncs_per_step,
                       "transport": "gloo (rehearsal)" if args.rehearse else "rccl"}
        res["check"] = check
    if world == 1:
        def rec_bytes(B):  # sum of the batch's record sizes (gaps excluded)
            return int(B.base.view(torch.int32)[(B.off // 4)].sum(dtype=torch.int64).item())

        # the fused fold's records == the step-by-step fold's (compacted, byte for byte)
        cf, cc = eng.orswot_compact(final, stream=stream), eng.orswot_compact(step_classic(), stream=stream)
        eng.status(stream)
        fold_equal = bool(cf.bytes == cc.bytes and torch.equal(cf.base[: cf.bytes], cc.base[: cc.bytes]))
        if not fold_equal:
            raise SystemExit("bench.py: the fused fold's records differ from the step-by-step fold's")
        del cf, cc

        # algorithmic bytes of the fold, from the real record sizes of every
        # step: merge k reads acc_k (replica 0, then the previous output) and
        # replica k+1, and writes its output; + 3 offsets per object-merge
        outs_b = [rec_bytes(o) for o in outs]
        alg_rec = sum(rec_bytes(B) for B in batches) + sum(outs_b) + sum(outs_b[:-1]) + 3 * 8 * n * (R - 1)
        # the roofline numerator: SURVEY.md §8(d)'s compact bytes of every merge's two inputs and output
        outs_c = [o.compact_bytes() for o in outs]
        in_c = sum(B.compact_bytes() for B in batches)
        alg = in_c + sum(outs_c) + sum(outs_c[:-1])
        ach = alg / (ev_ms * 1e-3) / 1e9
        ach_rec = alg_rec / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": f"crdt_orswot_fold: {R - 1} launches of orswot_sparse_mask_kernel "
                                                      "+ orswot_sparse_general_kernel", "achieved": ach,
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                           "kernel_ms": ev_ms, "alg_bytes_per_fold": alg, "merges_per_fold": R - 1,
                           "alg_bytes_def": "SURVEY.md §8(d) compact bytes (CSR top = 4 + 12 nnz) of both inputs + "
                                            "output of every fold merge, no header / padding / offsets",
                           "traffic": wl_traffic(args, "orswot_csr", "orswot_sparse_mask_kernel", "orswot_sparse_general_kernel"),
                           "record_bytes": {"per_launch": alg_rec / (R - 1), "achieved": ach_rec,
                                            "frac": ach_rec / HBM_PEAK_GBS},
                           "fold_equals_merge_calls": fold_equal}
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_ffi

            m = min(args.cpu_sample // 10, n)
            sub = crdts_hip.generate_replicas(m, 2, threads=args.threads)
            th = cpu_threads(args)
            # oracle fold step r0 ⊔ r1 (decode untimed), same record form
            secs = oracle_ffi.orswot_bench(sub[0][0], sub[0][1], sub[1][0], sub[1][1], th)
            res["cpu_baseline"] = {"value": m / secs, "unit": "object-merges/s", "cores": th, "kind": "port", **cpu_cores_note(),
                                   "sample": f"{m} objects, replica 0 ⊔ replica 1, oracle merge loop, {th} threads"}
    return res


def run_gcounter_ae(args, rank, world, local, eng=None):
    """Config 4 (BASELINE.json configs[3]): 1B GCounters x 8 dense actor slots
    (64 GB of u64 per GPU); replica r increments slot r. At N > 1 a step is the
    in-place RCCL all-reduce(max) over xGMI (u64-exact; repeated steps are
    idempotent); after the timed steps every rank's digest of its 64 GB must be
    equal, and sampled rows must equal the max over every rank's pre-join rows.
    At N = 1 a step is the local join of two such replicas (dense_max_kernel)."""
    import torch
    import torch.distributed as dist

    import crdts_hip
    from crdts_hip import replica

    n = args.n_obj or 1_000_000_000
    A = 8
    dev = f"cuda:{local}"
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0FFEE04)
    base = torch.randint(0, 1 << 40, (n, A), dtype=torch.int64, device=dev, generator=g)
    g.manual_seed(0xC0FFEE04 + 1 + rank)
    mine_slot = rank % A
    base[:, mine_slot] += torch.randint(1, 1 << 20, (n,), dtype=torch.int64, device=dev, generator=g)
    eng = eng or crdts_hip.Engine(local)
    stream = torch.cuda.Stream(device=local)
    torch.cuda.synchronize()  # generated on torch's stream; the joins run on `stream`
    check = None
    if world > 1:
        if not args.rehearse and not eng.has_comm:
            replica.init_comm(eng)  # the context's own RCCL communicator (crdt_comm_init)
        # pre-join sample rows (head, middle, tail), every rank's, for the check
        m = min(4096, n)
        idx = torch.cat([torch.arange(0, m, device=dev), torch.arange(n // 2, n // 2 + m, device=dev) % n,
                         torch.arange(n - m, n, device=dev)])
        pre = base[idx].contiguous()
        parts = [torch.empty_like(pre) for _ in range(world)]
        dist.all_gather(parts, pre)
        expect = torch.stack(parts).amax(0)  # counters < 2^41: signed max == u64 max here
        del parts

        if args.rehearse:  # the product's all-reduce over the gloo transport (crdt_replica_allreduce_max_transport)
            T = replica.GlooTransport()
            flat_rows = base.view(-1)

            def step():
                eng.replica_allreduce_max_transport(flat_rows, T, stream=stream)
        else:
            def step():
                replica.dense_allreduce_max(base, engine=eng, stream=stream)
    else:
        other = base.clone()
        other[:, (mine_slot + 1) % A] += 1

        def step():
            eng.dense_merge(base, other, A, "gcounter", stream=stream)

    wall, ev_ms = _timed_steps(args, world, stream, step)
    bytes_per_gpu = 8 * n * A
    res = {
        "metric": "replica anti-entropy: GCounters joined/sec (node), 8 dense actors",
        "value": sum_over_ranks(float(n * args.steps), world) / wall, "unit": "objects/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: U[0,2^40) base + per-replica increments of its own slot",
        "config": {"workload": f"gcounter_ae config4 (BASELINE.json configs[3]): {n} GCounters x {A} slots per GPU",
                   "bytes_per_gpu": bytes_per_gpu,
                   "parallelism": ((f"all-reduce(max) over {world} ranks through the gloo transport "
                                    "(crdt_replica_allreduce_max_transport)") if args.rehearse else
                                   (f"RCCL all-reduce(max) over {world} GPUs, native u64 "
                                    "(crdt_replica_allreduce_max)")) if world > 1
                   else "local replica join (dense_max_kernel)"},
    }
    if world > 1:
        torch.cuda.synchronize()
        ok_sample = bool(torch.equal(base[idx], expect))
        dg = int(base.sum(dtype=torch.int64).item()) % (1 << 64)  # wraps mod 2^64: order-independent
        digests = [x[0] for x in _gather_ints([dg], world)]
        check = {"digests_equal": len(set(digests)) == 1, "digest": f"{dg:016x}", "sample_rows": int(idx.numel()),
                 "sample_ok": ok_sample, "ok": ok_sample and len(set(digests)) == 1}
        if not check["ok"]:
            print(f"bench.py rank {rank}: config-4 anti-entropy check FAILED: {check}", file=sys.stderr)
        # ring all-reduce bus bandwidth convention: 2 (N-1)/N x bytes / time
        res["comm"] = {"rccl_ranks": None if args.rehearse else eng.comm_count(),
                       "transport": "gloo (rehearsal)" if args.rehearse else "rccl",
                       "algbw_GBps": bytes_per_gpu / (ev_ms * 1e-3) / 1e9,
                       "busbw_GBps": 2 * (world - 1) / world * bytes_per_gpu / (ev_ms * 1e-3) / 1e9,
                       "xgmi_peak_GBps": 7 * 153}
        res["check"] = check
        # the owner-shard variant: reduce-scatter(max),
        # each rank keeps its 1/N of the joined counters (crdt_replica_reduce_scatter_max)
        flat = base.reshape(-1)[: (base.numel() // world) * world]
        if args.rehearse:  # the product's reduce-scatter over the gloo transport
            def rs_step():
                return eng.replica_reduce_scatter_max_transport(flat, T, stream=stream)
        else:
            def rs_step():
                return replica.dense_reduce_scatter_max(flat, engine=eng, stream=stream)
        _, rs_ms = _timed_steps(args, world, stream, rs_step)
        res["comm"]["reduce_scatter"] = {"ms": rs_ms, "algbw_GBps": bytes_per_gpu / (rs_ms * 1e-3) / 1e9,
                                         "busbw_GBps": (world - 1) / world * bytes_per_gpu / (rs_ms * 1e-3) / 1e9}
    else:
        ach = 3 * bytes_per_gpu / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "dense_max_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms,
                           "alg_bytes_per_launch": 3 * bytes_per_gpu, "traffic": None}
    return res


def run_clock_csr(args, rank, world, local):
    """Sparse (CSR) VClock / GCounter merge (SURVEY.md §8(a) A2 / A6 over a
    large actor universe; VClock::merge src/vclock.rs:131-137): 10M clock pairs
    per GPU over a 1024-actor universe, ~48 actors per clock (one per band of
    18 ids, present with p = 6/7), the other side sharing 75 % of the actors,
    counters U[1, 2^40). A step = one crdt_vclock_csr_merge launch over the
    batch (inputs resident in HBM); spot parity against the oracle first."""
    import numpy as np
    import torch

    import crdts_hip

    n = args.n_obj or 10_000_000
    slots, universe = 56, 1024
    band = universe // slots
    dev = f"cuda:{local}"
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0FFEE09 + rank)
    js = torch.randint(0, band, (n, slots), dtype=torch.int32, device=dev, generator=g)
    jo = torch.where(torch.rand((n, slots), device=dev, generator=g) < 0.75, js,
                     torch.randint(0, band, (n, slots), dtype=torch.int32, device=dev, generator=g))
    base = torch.arange(slots, dtype=torch.int32, device=dev)[None, :] * band
    sides = []
    for j in (js, jo):
        present = torch.rand((n, slots), device=dev, generator=g) < 6 / 7
        act = (base + j)[present].contiguous()
        ln = present.sum(1, dtype=torch.int32)
        off = torch.cumsum(ln, 0, dtype=torch.int64) - ln
        ctr = torch.randint(1, 1 << 40, (act.numel(),), dtype=torch.int64, device=dev, generator=g)
        sides.append(crdts_hip.ClockBatch(off, ln, act, ctr))
        del present
    del js, jo
    S, O = sides
    eng = crdts_hip.Engine(local)
    stream = torch.cuda.Stream(device=local)
    torch.cuda.synchronize()  # the batches were generated on torch's stream; the merges run on `stream`
    out = eng.clock_csr_merge(S, O, stream=stream)  # checked launch
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi

    m = 2000  # spot parity (the first m objects, re-based)
    def head(B):
        o = B.off[:m].cpu().numpy().view(np.uint64)
        ln = B.len[:m].cpu().numpy().view(np.uint32)
        e = int(o[-1]) + int(ln[-1])
        return o, ln, B.act[:e].cpu().numpy().view(np.uint32), B.ctr[:e].cpu().numpy().view(np.uint64)
    eo, el, ea, ec = oracle_ffi.vclock_csr_merge(head(S), head(O))
    go, gl, ga, gc = out.off[:m].cpu().numpy().view(np.uint64), out.len[:m].cpu().numpy().view(np.uint32), None, None
    assert (go == eo).all() and (gl == el).all(), "clock_csr spot parity: placement / lengths"
    hact = out.act[: int(eo[-1]) + int(el[-1])].cpu().numpy().view(np.uint32)
    hctr = out.ctr[: int(eo[-1]) + int(el[-1])].cpu().numpy().view(np.uint64)
    for o_, l_ in zip(eo.tolist(), el.tolist()):
        assert (hact[o_:o_ + l_] == ea[o_:o_ + l_]).all() and (hctr[o_:o_ + l_] == ec[o_:o_ + l_]).all()

    def step():
        eng.clock_csr_merge(S, O, out=out, stream=stream, check_status=False)

    wall, ev_ms = _timed_steps(args, world, stream, step)
    eng.status(stream)
    nnz_s, nnz_o = S.n_entries, O.n_entries
    nnz_u = int(out.len.sum(dtype=torch.int64).item())
    alg = 12 * (nnz_s + nnz_o + nnz_u) + 3 * 12 * n  # entries read / written + (off, len) per object and side
    ach = alg / (ev_ms * 1e-3) / 1e9
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "sparse (CSR) VClock merges/sec (node), 1024-actor universe",
        "value": total / wall, "unit": "merges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic: ~48 of 1024 actors per clock, 75 % shared across the pair, U[1,2^40)",
        "config": {"workload": f"clock_csr: {n} CSR clock pairs per GPU, universe {universe}, "
                               f"{nnz_s / n:.1f} + {nnz_o / n:.1f} -> {nnz_u / n:.1f} entries",
                   "parallelism": f"dp{world} (objects sharded)"},
    }
    if world == 1:
        res["roofline"] = {"bound": "hbm", "kernel": "clock_csr_merge_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms, "alg_bytes_per_launch": alg,
                           "traffic": wl_traffic(args, "clock_csr", "clock_csr_merge_kernel")}
        if not args.no_cpu_baseline:
            mm = min(args.cpu_sample, n)
            th = cpu_threads(args)

            def headm(B):
                o = B.off[:mm].cpu().numpy().view(np.uint64)
                ln = B.len[:mm].cpu().numpy().view(np.uint32)
                e = int(o[-1]) + int(ln[-1])
                return o, ln, B.act[:e].cpu().numpy().view(np.uint32), B.ctr[:e].cpu().numpy().view(np.uint64)
            secs = oracle_ffi.vclock_csr_bench(headm(S), headm(O), th)
            res["cpu_baseline"] = {"value": mm / secs, "unit": "merges/s", "cores": th, "kind": "port",
                                   **cpu_cores_note(),
                                   "sample": f"first {mm} clock pairs, VClock::merge over std::map (decode untimed), "
                                             f"{th} threads"}
    return res


def run_truncate(args, rank, world, local):
    """Batched Causal::truncate for Orswot (src/orswot.rs:159-172) over the
    config-3 shard: record i truncated by a clock derived from its own top
    clock T — c[x] = T[x] - 2 for even actors, T[x] for actors 1 mod 4, absent
    otherwise — so about a third of the member bytes and some top-clock entries
    are dropped (config-3 dots sit within a few counts of T). A step = one crdt_orswot_truncate launch (inputs
    resident in HBM); spot parity against the oracle first."""
    import ctypes as C

    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip._lib import check, lib

    n = args.n_obj or 1_000_000
    A = 16
    (lb, lo), _ = crdts_hip.generate_orswot(n, first_obj=rank * n, threads=args.threads)
    top = lb[: lb.nbytes // 8 * 8].view(np.uint64)[(lo // 8 + 4)[:, None] + np.arange(A, dtype=np.uint64)[None, :]]
    x = np.arange(A)
    cut_at = np.where(x % 2 == 0, np.where(top > 2, top - 2, 0), np.where(x % 4 == 1, top, 0)).astype(np.uint64)
    present = cut_at > 0
    act = np.nonzero(present)[1].astype(np.uint32)
    ctr = cut_at[present].astype(np.uint64)
    ln = present.sum(1).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    del top, cut_at, present
    eng = crdts_hip.Engine(local)
    B = crdts_hip.OrswotBatch.from_host(lb, lo, A, device=local)
    K = crdts_hip.ClockBatch.from_host(coff, ln, act, ctr, device=local)
    stream = torch.cuda.Stream(device=local)
    torch.cuda.synchronize()
    out = eng.orswot_truncate(B, K, stream=stream)  # checked launch; its buffers are reused below
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi

    m = min(2000, n)  # spot parity: the first m records
    e_end = int(coff[m - 1]) + int(ln[m - 1])
    cut = int(lo[m]) if n > m else lb.nbytes
    eb, eo = oracle_ffi.orswot_truncate_batch(lb[:cut], lo[:m], (coff[:m], ln[:m], act[:e_end], ctr[:e_end]), A)
    got = crdts_hip.OrswotBatch(out.base, out.off[:m], A).records()
    for i in range(m):
        sz = int(np.frombuffer(eb[int(eo[i]):int(eo[i]) + 4].tobytes(), np.uint32)[0])
        assert got[i] == eb[int(eo[i]):int(eo[i]) + sz].tobytes(), f"truncate spot parity, object {i}"
    st = C.c_void_p(stream.cuda_stream)
    bt, ct = B.cbatch(), K.cstruct()

    def step():
        check(lib.crdt_orswot_truncate(eng.ctx, C.byref(bt), C.byref(ct), A, 0, C.c_void_p(out.base.data_ptr()),
                                       C.c_void_p(out.off.data_ptr()), int(out.base.numel()), st))

    wall, ev_ms = _timed_steps(args, world, stream, step)
    eng.status(stream)
    out_sizes = out.base.view(torch.int32)[(out.off // 4)].cpu().numpy().astype(np.int64)
    alg = int(lb.nbytes) + int(out_sizes.sum()) + 12 * int(ln.sum()) + n * (8 + 8 + 4 + 8)
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "batched Orswot::truncate objects/sec (node)", "value": total / wall, "unit": "objects/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: config-3 op-simulated Orswots, each truncated by a clock derived from its top clock",
        "config": {"workload": f"truncate config3: {n} objects per GPU, {ln.mean():.1f}-entry clocks, "
                               f"{out_sizes.mean():.0f} B of {lb.nbytes / n:.0f} B kept per record",
                   "parallelism": f"dp{world} (objects sharded)"},
    }
    if world == 1:
        ach = alg / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "orswot_truncate_fast_kernel (+ orswot_truncate_kernel for the records it lists)",
                           "achieved": ach, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms, "alg_bytes_per_launch": alg,
                           "traffic": wl_traffic(args, "truncate", "orswot_truncate_fast_kernel", "orswot_truncate_kernel")}
        if not args.no_cpu_baseline:
            mm = min(args.cpu_sample, n)
            th = cpu_threads(args)
            e2 = int(coff[mm - 1]) + int(ln[mm - 1])
            secs = oracle_ffi.orswot_truncate_bench(lb, lo[:mm], (coff[:mm], ln[:mm], act[:e2], ctr[:e2]), th)
            res["cpu_baseline"] = {"value": mm / secs, "unit": "objects/s", "cores": th, "kind": "port",
                                   **cpu_cores_note(),
                                   "sample": f"first {mm} objects, Orswot::truncate over the oracle's containers "
                                             f"(decode untimed), {th} threads"}
    return res


def run_spawn_check(args, rank, world, local):
    """CPU only (gloo): what the launch path gives each rank — its rank, the
    world size, LOCAL_RANK (the GPU it would bind) and its pid — all-gathered."""
    import torch
    import torch.distributed as dist

    me = torch.tensor([rank, world, local, os.getpid()], dtype=torch.int64)
    parts = [torch.empty_like(me) for _ in range(world)]
    if world > 1:
        dist.all_gather(parts, me)
    else:
        parts = [me]
    return {"metric": "spawn_check", "value": float(world), "unit": "ranks", "n_gpus": world,
            "ranks": [p.tolist() for p in parts]}


def run_bincode(args, rank, world, local):
    """ingest of the reference's binary form
    (`from_binary`, src/lib.rs:78-83) into canonical records, and egest
    (`to_binary`, :62-64), for the config-3 objects (1M per GPU, actors u8,
    members u64). A step = one ingest of the whole shard: record bounds from
    the blob lengths (crdt_orswot_bincode_record_bounds: no blob read), the
    offset scan and the decode pass — every blob is read once, records land
    in a gapped batch — inputs resident in HBM; egest is timed the same way
    and reported beside it."""
    import ctypes as C

    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip._lib import check, lib

    n = args.n_obj or 1_000_000
    WA, WM, A = 1, 8, 16
    (lb, lo), _ = crdts_hip.generate_orswot(n, first_obj=rank * n, threads=args.threads)
    eng = crdts_hip.Engine(local)
    dev = f"cuda:{local}"
    B = crdts_hip.OrswotBatch.from_host(lb, lo, A, device=local)
    blobs, boff, blen = eng.orswot_to_bincode(B, WA, WM)  # checked once; the timed steps reuse the buffers
    back = eng.orswot_from_bincode(blobs, boff, blen, A, WA, WM)
    assert torch.equal(back.base[: int(lb.nbytes)], B.base[: int(lb.nbytes)])
    stream = torch.cuda.Stream(device=local)
    st = C.c_void_p(stream.cuda_stream)
    sizes = torch.empty(n, dtype=torch.int64, device=dev)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    check(lib.crdt_orswot_bincode_record_bounds(eng.ctx, p(blen), n, WA, WM, A, 0, p(sizes), st))
    stream.synchronize()
    rec = torch.empty(int(sizes.sum().item()), dtype=torch.uint8, device=dev)
    roff = torch.empty(n, dtype=torch.int64, device=dev)

    def ingest():
        check(lib.crdt_orswot_bincode_record_bounds(eng.ctx, p(blen), n, WA, WM, A, 0, p(sizes), st))
        with torch.cuda.stream(stream):
            torch.cumsum(sizes, 0, out=roff)
            roff.sub_(sizes)
        check(lib.crdt_orswot_from_bincode(eng.ctx, p(blobs), int(blobs.numel()), p(boff), p(blen), n, WA, WM, A,
                                           0, p(rec), p(roff), int(rec.numel()), st))

    eb = B.cbatch()
    lens = torch.empty(n, dtype=torch.int64, device=dev)
    eoff = torch.empty(n, dtype=torch.int64, device=dev)
    eout = torch.empty_like(blobs)

    def egest():
        check(lib.crdt_orswot_bincode_sizes(eng.ctx, C.byref(eb), A, 0, WA, WM, p(lens), st))
        with torch.cuda.stream(stream):
            pad = (lens + 15) // 16 * 16
            torch.cumsum(pad, 0, out=eoff)
            eoff.sub_(pad)
        check(lib.crdt_orswot_to_bincode(eng.ctx, C.byref(eb), A, 0, WA, WM, p(eout), p(eoff), int(eout.numel()),
                                         st))

    wall, ev_ms = _timed_steps(args, world, stream, ingest)
    eng.status(stream)
    packed = eng.orswot_compact(crdts_hip.OrswotBatch(rec, roff, A, int(rec.numel())))  # gaps removed: the batch
    assert torch.equal(packed.base[: int(lb.nbytes)], B.base[: int(lb.nbytes)])
    ewall, eev_ms = _timed_steps(args, world, stream, egest)
    eng.status(stream)
    assert torch.equal(eout, blobs)
    blob_bytes = int(blen.sum().item())
    rec_bytes = int(lb.nbytes)
    # algorithmic bytes: ingest reads every blob once + offsets/lengths, writes every record
    # once + bounds/offsets; egest reads records twice (sizes pass, write pass), writes blobs once
    alg_in = blob_bytes + rec_bytes + 8 * 6 * n
    alg_eg = 2 * rec_bytes + blob_bytes + 8 * 5 * n
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "bincode ingest (from_binary -> canonical records) objects/sec (node)",
        "value": total / wall, "unit": "objects/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic: config-3 op-simulated Orswots, their to_binary form (actor u8, member u64)",
        "config": {"workload": f"bincode config3: {n} objects per GPU, {blob_bytes / n:.0f} B blob, "
                               f"{rec_bytes / n:.0f} B record", "parallelism": f"dp{world} (objects sharded)"},
        "egest": {"value": sum_over_ranks(float(n * args.steps), world) / ewall, "unit": "objects/s",
                  "ms_per_step": ewall / args.steps * 1e3, "achieved_GBps": alg_eg / (eev_ms * 1e-3) / 1e9},
    }
    if world == 1:
        ach = alg_in / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "bincode_decode_kernel (+ bincode_bounds_kernel, scan)",
                           "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                           "kernel_ms": ev_ms, "alg_bytes_per_launch": alg_in,
                           "traffic": wl_traffic(args, "bincode", "bincode_bounds_kernel", "bincode_decode_kernel"),
                           "parity": "unpinned by reference output (bincode 0.9 restated, DESIGN.md §5b)"}
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_ffi

            m = min(args.cpu_sample // 5, n)
            hb = blobs.cpu().numpy()
            ho = boff[:m].cpu().numpy().astype(np.uint64)
            hl = blen[:m].cpu().numpy().astype(np.uint64)
            th = cpu_threads(args)
            secs = oracle_ffi.bincode_ingest_bench(hb, ho, hl, WA, WM, A, 0, th)
            res["cpu_baseline"] = {"value": m / secs, "unit": "objects/s", "cores": th, "kind": "port", **cpu_cores_note(),
                                   "sample": f"{m} blobs, from_binary into map/unordered_map + record encode, "
                                             f"{th} threads"}
    return res


def _apply_ops(lb, lo, n):
    """8 ops per config-3 object (numpy, deterministic): fresh adds to new and
    existing members, a future-context remove that a later add releases
    (apply_deferred), read-context removes that drop an entry / a dot."""
    import numpy as np

    C = np.uint64(1 << 33)
    i = np.arange(n, dtype=np.uint64)
    a = (i % np.uint64(16)).astype(np.uint32)
    b = ((i + np.uint64(5)) % np.uint64(16)).astype(np.uint32)
    hdr = lb[(lo[:, None].astype(np.int64) + np.arange(32)[None, :])].view(np.uint32).reshape(n, 8)
    nm = hdr[:, 2].astype(np.int64)
    key0 = lo.astype(np.int64) + 160
    k0 = np.where(nm > 0, lb[key0[:, None] + np.arange(8)[None, :]].view(np.uint64).ravel(), np.uint64(11))
    kmid = lo.astype(np.int64) + 160 + 8 * (nm // 2)
    k1 = np.where(nm > 0, lb[kmid[:, None] + np.arange(8)[None, :]].view(np.uint64).ravel(), np.uint64(13))
    new1 = (i * np.uint64(0x9E3779B97F4A7C15)) | np.uint64(1 << 63)
    new2 = new1 ^ np.uint64(0x5555)
    z = np.zeros(n, np.uint64)
    # op table: (kind, member, actor, counter, rm-clock actor, rm-clock counter)
    table = [(0, new1, a, C + np.uint64(1)), (0, k0, b, C + np.uint64(2)), (1, k1, a, C + np.uint64(5)),
             (0, k1, a, C + np.uint64(3)), (0, new2, a, C + np.uint64(5)), (1, new1, a, C + np.uint64(1)),
             (0, k0, b, C + np.uint64(6)), (1, k0, b, C + np.uint64(6))]
    K = len(table)
    kind = np.empty((n, K), np.uint32)
    mem = np.empty((n, K), np.uint64)
    act = np.zeros((n, K), np.uint32)
    ctr = np.zeros((n, K), np.uint64)
    npair = np.zeros((n, K), np.uint64)
    cact, cctr = [], []
    for j, (k, m, x, c) in enumerate(table):
        kind[:, j] = k
        mem[:, j] = m
        if k == 0:
            act[:, j] = x
            ctr[:, j] = c
        else:
            npair[:, j] = 1
            cact.append(x)
            cctr.append(c)
    rm_cols = [j for j, t in enumerate(table) if t[0] == 1]
    ca = np.zeros((n, K), np.uint32)
    cc = np.zeros((n, K), np.uint64)
    for col, x, c in zip(rm_cols, cact, cctr):
        ca[:, col] = x
        cc[:, col] = c
    sel = npair.ravel() > 0
    clk_act = ca.ravel()[sel]
    clk_ctr = cc.ravel()[sel]
    clk_end = np.cumsum(npair.ravel()).astype(np.uint64)
    obj_end = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(K))
    del z
    return obj_end, kind.ravel(), mem.ravel(), act.ravel(), ctr.ravel(), clk_end, clk_act, clk_ctr


def run_apply(args, rank, world, local):
    """the batched op path (CmRDT::apply for Orswot,
    src/orswot.rs:61-85) over the config-3 shard, 8 ops per object (adds,
    deferred and read-context removes, deferred releases). A step = one
    crdt_orswot_apply launch over all objects, inputs resident in HBM."""
    import ctypes as C

    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip._lib import Ops, check, lib

    n = args.n_obj or 1_000_000
    A = 16
    (lb, lo), _ = crdts_hip.generate_orswot(n, first_obj=rank * n, threads=args.threads)
    ops_np = _apply_ops(lb, lo, n)
    eng = crdts_hip.Engine(local)
    dev = f"cuda:{local}"
    B = crdts_hip.OrswotBatch.from_host(lb, lo, A, device=local)

    def t64(x):
        return torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev)

    def t32(x):
        return torch.from_numpy(np.ascontiguousarray(x).view(np.int32)).to(dev)

    o_end, kind, mem, act, ctr, cend, cact, cctr = ops_np
    ops = crdts_hip.OrswotOps(t64(o_end), t32(kind), t64(mem), t32(act), t64(ctr), t64(cend), t32(cact), t64(cctr))
    first = eng.orswot_apply(B, ops)  # checked launch; reused buffers below
    out, ooff = first.base, first.off
    n_ops, n_clk = ops.n_ops, ops.n_clk
    # spot parity against the oracle's op path on a sample
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi

    import records as R

    got = first.records()[:300]
    for i in range(300):
        o = oracle_ffi.OracleOrswot.decode(bytes(lb[lo[i]:lo[i] + int(np.frombuffer(lb[lo[i]:lo[i] + 4], np.uint32)[0])]))
        for q in range(int(o_end[i - 1]) if i else 0, int(o_end[i])):
            if kind[q] == 0:
                o.apply_add(int(act[q]), int(ctr[q]), int(mem[q]))
            else:
                b0 = int(cend[q - 1]) if q else 0
                o.apply_rm(int(mem[q]), [(int(cact[k]), int(cctr[k])) for k in range(b0, int(cend[q]))])
        assert o.encode(A) == got[i], f"apply parity, object {i}: {R.decode(got[i])}"
    stream = torch.cuda.Stream(device=local)
    st = C.c_void_p(stream.cuda_stream)
    bt = B.cbatch()
    co = ops.cops()

    def step():
        check(lib.crdt_orswot_apply(eng.ctx, C.byref(bt), C.byref(co), A, 0, C.c_void_p(out.data_ptr()),
                                    C.c_void_p(ooff.data_ptr()), int(out.numel()), st))

    wall, ev_ms = _timed_steps(args, world, stream, step)
    eng.status(stream)
    out_sizes = out.view(torch.int32)[(ooff // 4)].cpu().numpy().astype(np.int64)
    alg = int(lb.nbytes) + int(out_sizes.sum()) + n_ops * (4 + 8 + 4 + 8 + 8) + n_clk * 12 + 8 * 3 * n
    total = sum_over_ranks(float(n_ops * args.steps), world)
    res = {
        "metric": "batched Orswot op apply (CmRDT::apply) ops/sec (node)", "value": total / wall, "unit": "ops/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: config-3 op-simulated Orswots + 8 generated ops each (adds, deferred / read-ctx removes)",
        "config": {"workload": f"apply config3: {n} objects x {n_ops // n} ops per GPU",
                   "parallelism": f"dp{world} (objects sharded)"},
    }
    if world == 1:
        ach = alg / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "orswot_apply_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms, "alg_bytes_per_launch": alg,
                           "traffic": wl_traffic(args, "apply", "orswot_apply_kernel")}
        if not args.no_cpu_baseline:
            m = min(args.cpu_sample // 5, n)
            th = cpu_threads(args)
            sub = (o_end[:m], kind[:8 * m], mem[:8 * m], act[:8 * m], ctr[:8 * m], cend[:8 * m],
                   cact[:int(cend[8 * m - 1])], cctr[:int(cend[8 * m - 1])])
            secs = oracle_ffi.orswot_apply_bench(lb, lo[:m].astype(np.uint64), sub, th)
            res["cpu_baseline"] = {"value": 8 * m / secs, "unit": "ops/s", "cores": th, "kind": "port", **cpu_cores_note(),
                                   "sample": f"{m} objects x 8 ops, oracle op path (std::map/unordered_map), "
                                             f"{th} threads"}
    return res


def run_mvreg(args, rank, world, local):
    """batched MVReg<u64, A>::merge (src/mvreg.rs:121-153)
    over 4M registers per GPU (A = 16 dense actors, 4 (clock, value) slots per
    side, 8 out), and VClock partial_cmp (src/vclock.rs:59-71) over 100M row
    pairs reported beside it. Inputs resident in HBM."""
    import time as _t

    import numpy as np
    import torch

    import crdts_hip

    n = args.n_obj or 4_000_000
    A, cap = 16, 4
    dev = f"cuda:{local}"
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0FFEE06 + rank)

    def slab():
        cnt = torch.randint(0, cap + 1, (n,), dtype=torch.int32, device=dev, generator=g)
        clk = torch.randint(0, 3, (n, cap, A), dtype=torch.int64, device=dev, generator=g)
        clk *= (torch.arange(cap, device=dev)[None, :, None] < cnt[:, None, None])
        val = torch.randint(0, 1 << 62, (n, cap), dtype=torch.int64, device=dev, generator=g)
        return cnt, clk, val

    S, O = slab(), slab()
    eng = crdts_hip.Engine(local)
    stream = torch.cuda.Stream(device=local)
    torch.cuda.synchronize()  # generated on torch's stream; the merges run on `stream`
    out = eng.mvreg_merge(S, O, A, stream=stream)
    torch.cuda.synchronize()
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi

    m = 2000  # spot parity
    hs = [t[:m].cpu().numpy() for t in S]
    ho = [t[:m].cpu().numpy() for t in O]
    en, ec, ev = oracle_ffi.mvreg_merge(hs[0].view(np.uint32), hs[1].view(np.uint64), hs[2].view(np.uint64),
                                        ho[0].view(np.uint32), ho[1].view(np.uint64), ho[2].view(np.uint64), A, 2 * cap)
    assert (out[0][:m].cpu().numpy().view(np.uint32) == en).all()
    assert (out[1][:m].cpu().numpy().view(np.uint64) == ec).all()

    def step():
        eng.mvreg_merge(S, O, A, stream=stream, check_status=False)

    wall, ev_ms = _timed_steps(args, world, stream, step)
    eng.status(stream)
    alg = 2 * n * (4 + cap * A * 8 + cap * 8) + n * (4 + 2 * cap * A * 8 + 2 * cap * 8)
    # partial_cmp beside it: 100M dense row pairs
    npc = 100_000_000 if world == 1 else 50_000_000
    ra = torch.randint(0, 3, (npc, A), dtype=torch.int64, device=dev, generator=g)
    rb = ra.clone()
    rb[: npc // 2] += torch.randint(0, 2, (npc // 2, A), dtype=torch.int64, device=dev, generator=g)
    pc = lambda: eng.vclock_partial_cmp(ra, rb, A, stream=stream)  # noqa: E731
    pwall, pev = _timed_steps(args, world, stream, pc)
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "MVReg merges/sec (node)", "value": total / wall, "unit": "merges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: random MVRegs, 0-4 slots per side, 16 dense actors, counters U[0,3)",
        "config": {"workload": f"mvreg: {n} MVReg<u64> merges per GPU, A=16, 4+4 -> 8 slots",
                   "parallelism": f"dp{world} (objects sharded)"},
        "partial_cmp": {"value": sum_over_ranks(float(npc * args.steps), world) / pwall, "unit": "pairs/s",
                        "achieved_GBps": (2 * npc * A * 8 + npc) / (pev * 1e-3) / 1e9, "kernel_ms": pev},
    }
    if world == 1:
        ach = alg / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "mvreg_merge_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms, "alg_bytes_per_launch": alg,
                           "traffic": wl_traffic(args, "mvreg", "mvreg_merge_kernel")}
        if not args.no_cpu_baseline:
            mm = 200_000
            hs = [t[:mm].cpu().numpy() for t in S]
            ho = [t[:mm].cpu().numpy() for t in O]
            t0 = _t.perf_counter()
            oracle_ffi.mvreg_merge(hs[0].view(np.uint32), hs[1].view(np.uint64), hs[2].view(np.uint64),
                                   ho[0].view(np.uint32), ho[1].view(np.uint64), ho[2].view(np.uint64), A, 2 * cap)
            secs = _t.perf_counter() - t0
            res["cpu_baseline"] = {"value": mm / secs, "unit": "merges/s", "cores": 1, "kind": "port", **cpu_cores_note(),
                                   "sample": f"{mm} MVReg merges, oracle (std::map clocks), 1 thread, "
                                             "incl. slab<->map conversion"}
    return res


def run_map(args, rank, world, local):
    """batched Map<u64, MVReg<u64, A>, A>::merge
    (src/map.rs:191-268) over 250k replica pairs per GPU built by op
    simulation (A = 16; per side <= 8 keys, 4 values per key, 8 deferred
    removes of <= 8 keys). A step = one crdt_map_mvreg_merge launch."""
    import time as _t

    import numpy as np
    import torch

    import crdts_hip

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi

    n = args.n_obj or 250_000
    A, caps = 16, (8, 4, 8, 8)
    L, R = oracle_ffi.map_generate(0xC0FFEE07 + rank, n, A, 8, 12, caps)
    eng = crdts_hip.Engine(local)
    dev = f"cuda:{local}"
    dL, dR = L.to(dev), R.to(dev)
    out = eng.map_mvreg_merge(dL, dR, A)
    m = 2000
    sub = lambda S: crdts_hip.MapSlab({f: v[:m] for f, v in S.a.items()}, S.kcap, S.mcap, S.dcap, S.scap)  # noqa: E731
    exp = oracle_ffi.map_merge(sub(L), sub(R), A)
    got, exp = sub(out.host()).canonical(), exp.canonical()
    for f in exp.a:
        assert (got.a[f] == exp.a[f]).all(), f"map merge parity: {f}"
    stream = torch.cuda.Stream(device=local)

    def step():  # into the same output slab every step (the merge writes only its used slots)
        eng.map_mvreg_merge(dL, dR, A, stream=stream, check_status=False, out=out)

    wall, ev_ms = _timed_steps(args, world, stream, step)
    eng.status(stream)
    # algorithmic bytes: the states' used slots, not the slabs' capacity
    alg = L.used_bytes() + R.used_bytes() + out.used_bytes()
    cap_bytes = sum(int(v.numel()) * v.element_size() for S in (dL, dR, out) for v in S.a.values())
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "Map<u64, MVReg> merges/sec (node)", "value": total / wall, "unit": "merges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: op-simulated Map<u64, MVReg<u64>> replica pairs (updates, removes, deferred removes)",
        "config": {"workload": f"map: {n} map merges per GPU, A=16, caps {caps}",
                   "parallelism": f"dp{world} (objects sharded)", "slab_capacity_bytes": cap_bytes},
    }
    if world == 1:
        ach = alg / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "map_mvreg_merge_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms, "alg_bytes_per_launch": alg,
                           "traffic": wl_traffic(args, "map", "map_mvreg_merge_kernel")}
        if not args.no_cpu_baseline:
            mm = 20_000
            t0 = _t.perf_counter()
            oracle_ffi.map_merge(sub(L) if mm == m else crdts_hip.MapSlab({f: v[:mm] for f, v in L.a.items()}, *caps),
                                 crdts_hip.MapSlab({f: v[:mm] for f, v in R.a.items()}, *caps), A)
            secs = _t.perf_counter() - t0
            res["cpu_baseline"] = {"value": mm / secs, "unit": "merges/s", "cores": 1, "kind": "port", **cpu_cores_note(),
                                   "sample": f"{mm} map merges, oracle (std::map / BTreeMap-shaped), 1 thread, "
                                             "incl. slab<->map conversion"}
    return res


def run_map_map(args, rank, world, local):
    """Nested maps — the reference's TestMap, Map<u64, Map<u64, MVReg<u64>>>
    (test/map.rs:4-8; Map::merge src/map.rs:191-268 with the inner map's merge
    and truncate as the value's): batched crdt_map_map_merge over 200k
    replica pairs per GPU, A = 16, <= 4 outer and 4 inner keys per map. The
    pairs come from the op-path generator of the parity tests
    (tests/nested_gen.py: nested puts, outer and inner removes through read
    contexts, early third-replica removes left deferred, partial out-of-order
    exchange): 10k distinct pairs, tiled. A step = one crdt_map_map_merge
    (two launches: outer pass, inner merges with the truncation fused)."""
    import random
    import time as _t

    import numpy as np
    import torch

    import crdts_hip

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import map_slab
    import nested_gen

    n = args.n_obj or 200_000
    A, caps, inner = 16, dict(kcap=4, dcap=8, scap=4), (4, 8, 8, 4)
    n0 = min(n, 10_000)
    rng = random.Random(0xC0FFEE09 + rank)
    pairs = [nested_gen.pair(rng, list(range(A))) for _ in range(n0)]
    L0 = crdts_hip.MapMapSlab.alloc(n0, A, inner_caps=inner, **caps)
    R0 = crdts_hip.MapMapSlab.alloc(n0, A, inner_caps=inner, **caps)
    for i, (x, y) in enumerate(pairs):
        map_slab.nested_map_to_row(x, L0, i, A)
        map_slab.nested_map_to_row(y, R0, i, A)
    reps = -(-n // n0)

    def tile(S):
        t = lambda v: np.concatenate([v] * reps)[: n * (v.shape[0] // n0)]  # noqa: E731
        return crdts_hip.MapMapSlab({f: t(v) for f, v in S.a.items()}, S.kcap, S.dcap, S.scap,
                                    crdts_hip.MapSlab({f: t(v) for f, v in S.inner.a.items()}, *S.inner_caps))

    L, R = tile(L0), tile(R0)
    eng = crdts_hip.Engine(local)
    dev = f"cuda:{local}"
    dL, dR = L.to(dev), R.to(dev)
    out = eng.map_map_merge(dL, dR, A)
    h = out.host()
    for i in range(0, n0, max(1, n0 // 500)):  # parity on a sample: the restatement's merge
        exp = pairs[i][0].clone()
        exp.merge(pairs[i][1])
        assert map_slab.nested_map_from_row(h, i) == exp, f"nested map merge parity: pair {i}"
    stream = torch.cuda.Stream(device=local)

    def step():  # into the same output slabs every step (the merge writes only its used slots)
        eng.map_map_merge(dL, dR, A, stream=stream, check_status=False, out=out)

    wall, ev_ms = _timed_steps(args, world, stream, step)
    eng.status(stream)
    alg = L.used_bytes() + R.used_bytes() + out.used_bytes()
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "nested Map<u64, Map<u64, MVReg>> merges/sec (node)", "value": total / wall, "unit": "merges/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": f"synthetic: {n0} op-simulated TestMap replica pairs (tests/nested_gen.py), tiled to {n}",
        "config": {"workload": f"map_map: {n} nested map merges per GPU, A={A}, outer caps {caps}, inner caps {inner}",
                   "parallelism": f"dp{world} (objects sharded)"},
    }
    if world == 1:
        ach = alg / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "map_map_outer_kernel + map_mvreg_merge_kernel (tasks, "
                           "truncation fused)", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms, "alg_bytes_per_launch": alg,
                           "alg_bytes_def": "the used slots of both inputs and the output, outer and nested",
                           "traffic": wl_traffic(args, "map_map", "map_map_outer_kernel", "map_mvreg_merge_kernel")}
        if not args.no_cpu_baseline:
            import oracle_ffi

            th = cpu_threads(args)
            mm = min(n, 200_000)  # the tiled host slabs: the same pairs the GPU merged
            Ls, Rs = (crdts_hip.MapMapSlab({f: v[: mm * (v.shape[0] // n)] for f, v in S.a.items()}, S.kcap, S.dcap,
                                           S.scap, crdts_hip.MapSlab({f: v[: mm * (v.shape[0] // n)]
                                                                       for f, v in S.inner.a.items()}, *S.inner_caps))
                      for S in (L, R))
            secs = oracle_ffi.map_map_bench(Ls, Rs, A, th)
            res["cpu_baseline"] = {"value": mm / secs, "unit": "merges/s", "cores": th, "kind": "port",
                                   **cpu_cores_note(),
                                   "sample": f"{mm} nested map merges, the C++ restatement (oracle/ref_cpu.cpp "
                                             f"MapT<MapT<MVRegO>>, std::map containers), {th} threads, decode untimed"}
    return res


def run_map_orswot(args, rank, world, local):
    """SURVEY.md §8(f) rank 3 as written: batched Map<u64, Orswot<u64, A>, A>::merge
    (src/map.rs:192-269, nested Orswot::merge / truncate src/orswot.rs:87-172)
    over 100k replica pairs per GPU built by op simulation (A = 16; per side
    <= 8 keys of <= 8 members, 4 nested deferred removes, 8 map deferred
    removes). A step = one crdt_map_orswot_merge launch."""
    import time as _t

    import torch

    import crdts_hip

    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi

    n = args.n_obj or 100_000
    A = 16
    caps = dict(kcap=8, mcap=8, vdcap=4, vscap=4, dcap=8, scap=8)
    L, R = oracle_ffi.map_orswot_generate(0xC0FFEE08 + rank, n, A, 6, 8, 12, 20, caps)
    eng = crdts_hip.Engine(local)
    dev = f"cuda:{local}"
    dL, dR = L.to(dev), R.to(dev)
    out = eng.map_orswot_merge(dL, dR, A)
    m = 2000
    sub = lambda S, k: crdts_hip.MapOrswotSlab({f: v[:k] for f, v in S.a.items()}, S.caps)  # noqa: E731
    exp = oracle_ffi.map_orswot_merge(sub(L, m), sub(R, m), A)
    got = sub(out.host(), m).canonical()
    exp = exp.canonical()
    for f in exp.a:
        assert (got.a[f] == exp.a[f]).all(), f"map-orswot merge parity: {f}"
    stream = torch.cuda.Stream(device=local)

    def step():  # into the same output slab every step (the merge writes only its used slots)
        eng.map_orswot_merge(dL, dR, A, stream=stream, check_status=False, out=out)

    wall, ev_ms = _timed_steps(args, world, stream, step)
    eng.status(stream)
    # algorithmic bytes: the states' used slots (read both inputs, write the
    # output), not the slabs' capacity
    alg = L.used_bytes() + R.used_bytes() + out.used_bytes()
    cap_bytes = sum(int(v.numel()) * v.element_size() for S in (dL, dR, out) for v in S.a.values())
    total = sum_over_ranks(float(n * args.steps), world)
    res = {
        "metric": "Map<u64, Orswot> merges/sec (node)", "value": total / wall, "unit": "merges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: op-simulated Map<u64, Orswot<u64>> replica pairs (nested adds / removes, map removes, "
                "deferred removes at both levels)",
        "config": {"workload": f"map_orswot: {n} map merges per GPU, A=16, caps {caps}",
                   "parallelism": f"dp{world} (objects sharded)", "slab_capacity_bytes": cap_bytes},
    }
    if world == 1:
        ach = alg / (ev_ms * 1e-3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "map_orswot_merge_kernel", "achieved": ach,
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "kernel_ms": ev_ms,
                           "alg_bytes_per_launch": alg,
                           "traffic": wl_traffic(args, "map_orswot", "map_orswot_merge_kernel")}
        if not args.no_cpu_baseline:
            mm = 10_000
            t0 = _t.perf_counter()
            oracle_ffi.map_orswot_merge(sub(L, mm), sub(R, mm), A)
            secs = _t.perf_counter() - t0
            res["cpu_baseline"] = {"value": mm / secs, "unit": "merges/s", "cores": 1, "kind": "port",
                                   **cpu_cores_note(),
                                   "sample": f"{mm} map merges, oracle (BTreeMap / HashMap-shaped containers), "
                                             "1 thread, incl. slab<->map conversion"}
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))  # before any GPU call in this process
    rank, world, local = dist_setup(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if args.workload == "spawn_check":
        res = run_spawn_check(args, rank, world, local)
    elif args.workload in ("orswot", "orswot_tail", "orswot_csr_tail"):
        res = run_orswot(args, rank, world, local)
    elif args.workload == "vclock":
        res = run_vclock(args, rank, world, local)
    elif args.workload == "orswot_csr":
        res = run_orswot_csr(args, rank, world, local)
    elif args.workload == "gcounter_ae":
        res = run_gcounter_ae(args, rank, world, local)
    elif args.workload == "bincode":
        res = run_bincode(args, rank, world, local)
    elif args.workload == "apply":
        res = run_apply(args, rank, world, local)
    elif args.workload == "mvreg":
        res = run_mvreg(args, rank, world, local)
    elif args.workload == "map":
        res = run_map(args, rank, world, local)
    elif args.workload == "map_orswot":
        res = run_map_orswot(args, rank, world, local)
    elif args.workload == "map_map":
        res = run_map_map(args, rank, world, local)
    elif args.workload == "clock_csr":
        res = run_clock_csr(args, rank, world, local)
    elif args.workload == "truncate":
        res = run_truncate(args, rank, world, local)
    else:
        res = run_dense(args, rank, world, local, args.workload)
    failed = [k for k, v in res.get("anti_entropy", {}).items() if not (v.get("check") or {}).get("ok", True)]
    if not (res.get("check") or {}).get("ok", True):
        failed.append(args.workload)
    if rank == 0:
        if args.workload != "spawn_check":
            import crdts_hip

            res["build"] = crdts_hip.build_record()  # the library this run loaded, vs __graft_entry__.build()'s record
        if SETTLE:
            res["settle"] = dict(SETTLE)
        _emit(res)
    if failed:
        raise SystemExit(f"bench.py rank {rank}: cross-rank check failed: {failed}")
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
