#!/usr/bin/env python3
"""All-sources SPF throughput + buildRouteDb latency on the 10k-node grid.

Workload (BASELINE.json configs[1]): the benchmark grid
createGrid(n=100, 1 prefix, SP_ECMP) of RoutingBenchmarkUtils.cpp:271-313,
N = 10,000 nodes, E = 39,600 directed adjacencies, unit metrics. One sweep is
LinkState::runSpf from every node (dist row + ECMP first-hop mask row per
source, written to HBM) with the CSR mirror already resident in HBM.

A step (--scaling):
  whatif (default)  a fixed batch of --topologies what-if variants of the grid
                    (variant 0 the grid itself, variant t > 0 the grid with one
                    seeded link drained), every one swept from all 10,000
                    sources; the variants are split over the ranks (strong
                    scaling: total work fixed, no data-path collective), and a
                    rank deals its variants over --lanes contexts (one HIP
                    stream each) so independent sweeps overlap on the GPU
  strong            one topology, its 10,000 sources split into contiguous
                    degree-weighted blocks over the ranks
  weak              every rank sweeps all sources of its own variant
With --gpus N the driver starts one process per GPU (torch.distributed.run);
the only cross-rank traffic is the barrier and the max-over-ranks time.

Also reported: buildRouteDb("1") ms (cold: right after a topology-changing
adjacency update, so it includes the device mirror patch and the SPF; warm:
memoized SPF), the dominant kernels' HBM roofline figures, and the CPU oracle
(a port of the reference algorithm with its data structures) timed on a
bounded sample of the same workload on this host.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from openr_amd.sharding import dist_env, shard_sources  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--grid", type=int, default=100)
    p.add_argument("--scaling", choices=("whatif", "strong", "weak"), default="whatif")
    p.add_argument("--topologies", type=int, default=32,
                   help="what-if variants per step (--scaling whatif)")
    # 2 lanes: 22.9-23.0 ms per step against 23.0-23.1 at 3 and 23.6-23.8 at 4
    # on the round-5 kernels (profiles/r05/zh_lanes_ab.txt; 4 was best with the
    # round-3 kernels): two sweeps in flight already fill the CUs
    p.add_argument("--lanes", type=int, default=2,
                   help="stream lanes per rank: a rank's what-if variants are dealt over this many "
                        "contexts (own HIP stream each) so their sweeps overlap on the GPU")
    p.add_argument("--cpu-sample", type=int, default=256, help="oracle sources per thread config")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="oracle threads (0: every CPU this process may use)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--rehearse-on-one-gpu", action="store_true",
                   help="rehearsal of the N-rank path on a one-GPU box: every rank drives GPU 0 "
                        "and the ranks sync over gloo (never used for reported numbers)")
    p.add_argument("--no-route-db", action="store_true")
    p.add_argument("--legs", default="c1,c2w,c3,c4,c5",
                   help="extra BASELINE configs reported under 'legs' (c1,c2w,c3,c4,c5; '' for none)")
    return p.parse_args()


def drain_what_if_link(adj_dbs, n, rank):
    """Overload both adjacencies of one seeded grid link (a what-if failure);
    returns them (clear isOverloaded to undo)."""
    import random
    rng = random.Random(1000 + rank)
    db = adj_dbs[rng.randrange(n * n)]
    adj = db.adjacencies[rng.randrange(len(db.adjacencies))]
    adj.isOverloaded = True
    peer = adj_dbs[int(adj.otherNodeName)]
    for back in peer.adjacencies:
        if back.otherNodeName == db.thisNodeName:
            back.isOverloaded = True
            return [adj, back]
    return [adj]


def median_ms(fn, reps):
    return statistics.median(fn() for _ in range(reps))


def main():
    args = parse()
    rank, world, local = dist_env()
    if args.rehearse_on_one_gpu:
        local = 0
    os.environ.setdefault("ORH_DEVICE", str(local))  # before the host library opens a context
    # the deployment's allocator policy (opt-in, process-global: keep freed
    # route-DB pages in glibc's arenas)
    os.environ.setdefault("ORH_MALLOC_TUNE", "1")
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    if world > 1:
        if args.rehearse_on_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64,
                         device="cpu" if args.rehearse_on_one_gpu else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    from openr_amd import host_backend
    from openr_amd.facade import load_topology
    from openr_amd.sharding import degree_weighted_sources, shard_bounds
    from openr_amd.topology import bench_grid
    from openr_amd.types import K_TESTING_AREA

    n = args.grid
    names = [str(i) for i in range(n * n)]
    hip = host_backend()
    # (variant, sources) units of this rank
    if args.scaling == "whatif":
        T = max(1, args.topologies)
        lo, hi = shard_bounds(T, world, rank)
        units = [(t, names) for t in range(lo, hi)]
        total_units = T * n * n
    elif args.scaling == "strong":
        units = [(0, None)]  # sources picked below (degree-weighted block)
        total_units = n * n
    else:
        units = [(rank, names)]
        total_units = n * n * world
    sweeps, base = [], None
    adj_dbs, prefixes = bench_grid(n, 1)  # one grid; a variant drains a link while it loads
    for i, (t, srcs) in enumerate(units):
        drained = drain_what_if_link(adj_dbs, n, t) if t > 0 else []
        als, ps = load_topology(hip, adj_dbs, prefixes, lane=i % max(1, args.lanes))
        for adj in drained:
            adj.isOverloaded = False
        ls = als[K_TESTING_AREA]
        if srcs is None:
            degrees = [len(db.adjacencies) for db in adj_dbs]
            srcs = degree_weighted_sources(names, degrees, world, rank)
        sweeps.append((t, srcs, ls, ls._impl.sweep(srcs, True) if srcs else None))
        if t == 0:
            base = (adj_dbs, prefixes, als, ps, ls)

    def run_all():
        for _, _, _, sw in sweeps:
            if sw is not None:
                sw.run()  # asynchronous on the context stream

    def sync_all():
        for _, _, _, sw in sweeps:
            if sw is not None:
                sw.sync()

    for _ in range(args.warmup):
        run_all()
    sync_all()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_all()
    sync_all()
    torch.cuda.synchronize()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)

    # device time of one sweep's launches (HIP events on the sweep's own
    # stream), measured outside the timed region
    probe = next((sw for _, srcs, _, sw in sweeps if sw is not None and len(srcs) == n * n),
                 next((sw for *_, sw in sweeps if sw is not None), None))
    kernel_ms, phases = [], []
    step_plan = None
    if probe is not None:
        for _ in range(max(3, min(args.steps, 10))):
            probe.run()
            kernel_ms.append(probe.last_ms())
            phases.append(probe.phase_ms())
        probe_info = probe.info()
        # the same sweep alone on the plan the timed step's overlapping sweeps
        # run (8-wave batches: ORH_MS_BLOCK=512 turns the lone-sweep plan off)
        os.environ["ORH_MS_BLOCK"] = "512"
        try:
            sp_ms, sp_ph = [], []
            for _ in range(max(3, min(args.steps, 10))):
                probe.run()
                sp_ms.append(probe.last_ms())
                sp_ph.append(probe.phase_ms())
            step_plan = (statistics.mean(sp_ms), [round(statistics.mean(p[i] for p in sp_ph), 4) for i in (0, 1)],
                         probe.info())
        finally:
            del os.environ["ORH_MS_BLOCK"]

    value = total_units * args.steps / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # size-independent correctness check on the timed output: unit metrics,
    # so dist(src, v) is the Manhattan distance on the undrained grid
    import numpy as np
    rr, cc = np.divmod(np.arange(n * n), n)
    for t, srcs, ls, sw in sweeps:
        if t != 0 or sw is None:
            continue
        node_ids = {name: i for i, name in enumerate(ls._impl.node_names())}
        ids = np.array([node_ids[str(v)] for v in range(n * n)])
        for i in (0, len(srcs) // 2, len(srcs) - 1):
            s_ = int(srcs[i])
            dist_row, _ = sw.fetch(i)
            if not np.array_equal(dist_row[ids], np.abs(rr - rr[s_]) + np.abs(cc - cc[s_])):
                raise SystemExit(f"bench: wrong distances for source {s_}")

    # N ranks: rank r runs block r of the C3 prefix-sharded route build and
    # of the C4 what-if job / KSP2 batch on its own GPU (bench_legs.run_ranks);
    # rank 0 reports the max over ranks. Untimed by the step's clock.
    rank_legs = None
    if world > 1 and args.legs:
        import bench_legs
        mine = bench_legs.run_ranks(args.legs.split(","), hip, rank, world)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        rank_legs = bench_legs.merge_ranks(gathered, world)

    if rank != 0:
        barrier()
        return

    # roofline of the sweep: B = 4(N+1) + 8E + N(4D + 4W)
    N, E, W = probe.nodes, probe.edges, probe.words
    srcs_probe = probe.sources
    bytes_per_source = 4 * (N + 1) + 8 * E + N * (4 * 1 + 4 * W)
    per_launch = bytes_per_source * srcs_probe
    kms = statistics.mean(kernel_ms)
    achieved = per_launch / (kms * 1e-3) / 1e9
    out_bytes = srcs_probe * N * (4 + 4 * W)  # the dist + first-hop rows alone

    traffic, traffic_src = pmc_traffic()
    parallelism = {"whatif": f"{args.topologies} what-if variants split over {world} rank(s)",
                   "strong": f"one topology, sources in {world} degree-weighted block(s)",
                   "weak": f"{world} variant(s), one per rank"}[args.scaling]
    out = {
        "metric": "all-source SPF runs/sec + buildRouteDb ms on 10k-node topology",
        "value": round(value, 1),
        "unit": "SPF-sources/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.scaling == "weak" else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: reference benchmark grid generator (createGrid n=100)",
        "config": {"workload": f"C2 {n}x{n} grid all-sources SPF (N={N}, E={E})",
                   "step": (f"{args.topologies} x {n * n} sources" if args.scaling == "whatif"
                            else f"{total_units} sources"),
                   "parallelism": parallelism},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel_ms": round(kms, 4),
                     # the sweep ran alone: the lone-sweep plan (12-wave
                     # batches); the step's overlapping sweeps run 8-wave ones
                     "plan": {"ms_threads": probe_info.get("ms_threads"),
                              "batch_sources": probe_info.get("batch_sources")},
                     "phase_ms": [round(statistics.mean(p[0] for p in phases), 4),
                                  round(statistics.mean(p[1] for p in phases), 4)],
                     # the probe above runs the lone-sweep plan (nothing else in
                     # flight); the step's sweeps run this one
                     "step_plan_sweep": None if step_plan is None else {
                         "kernel_ms": round(step_plan[0], 4), "phase_ms": step_plan[1],
                         "ms_threads": step_plan[2].get("ms_threads"),
                         "achieved": round(per_launch / (step_plan[0] * 1e-3) / 1e9, 1),
                         "frac": round(per_launch / (step_plan[0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                     "algorithmic_bytes_per_source": bytes_per_source,
                     "sources_per_launch": srcs_probe,
                     "output_floor": {"bytes": out_bytes,
                                      "frac": round(out_bytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                     # the timed region as a whole: every sweep's algorithmic
                     # bytes over the wall time of a step (overlapping lanes)
                     "step": {"achieved": round(bytes_per_source * total_units / world / (ms_per_step * 1e-3) / 1e9, 1),
                              "frac": round(bytes_per_source * total_units / world / (ms_per_step * 1e-3) / 1e9
                                            / HBM_PEAK_GBS, 4),
                              "note": "per-GPU algorithmic bytes of one step / ms_per_step; 'achieved' above "
                                      "is one sweep launch alone (HIP events), as rocprof's kernel averages"}},
    }

    if not args.no_route_db and base is not None:
        adj_dbs, prefixes, als, ps, ls = base
        solver = hip.spf_solver("1", True)
        solver.build_route_db("1", als, ps)
        db = adj_dbs[n * n // 2]
        flips = [0]

        def cold():
            flips[0] ^= 1  # topology change: memo cleared, mirror patched
            db.adjacencies[0].metric = 1 + flips[0]
            ls.update_adjacency_database(db)
            return profiled_build(solver._impl, "1", als._impl, ps._impl)

        def warm():
            return profiled_build(solver._impl, "1", als._impl, ps._impl)

        # two untimed topology changes first: the first ones after the initial
        # build grow one-time buffers (mirror patch staging, set caches) and
        # measured 3.5-4.4 ms against a steady 2.3-2.7 (tools/c2_build_spread.py)
        cold()
        cold()
        st0 = cgroup_cpu_stat()
        cold_runs = [cold() for _ in range(7)]
        st1 = cgroup_cpu_stat()
        warm_runs = [warm() for _ in range(7)]
        st2 = cgroup_cpu_stat()
        cold_ms = [r["ms"] for r in cold_runs]
        warm_ms = [r["ms"] for r in warm_runs]
        out["build_route_db_ms"] = round(statistics.median(cold_ms), 3)
        out["build_route_db_warm_ms"] = round(statistics.median(warm_ms), 3)
        out["build_route_db_runs"] = {"cold_ms": spread(cold_ms), "warm_ms": spread(warm_ms),
                                      "cold_settle": "2 untimed topology-change builds before the 7 timed ones",
                                      "phases": {"cold": phase_summary(cold_runs),
                                                 "warm": phase_summary(warm_runs)},
                                      "host_pool_threads": hip.module.host_threads(),
                                      "cgroup_throttling": {"cold": throttle_delta(st0, st1),
                                                            "warm": throttle_delta(st1, st2)}}
        db.adjacencies[0].metric = 1
        ls.update_adjacency_database(db)

    if world == 1 and not args.no_cpu_baseline and base is not None:
        out.update(cpu_baseline(args, base[0], base[1], n, value))
    if world == 1 and args.legs:
        import bench_legs
        out["legs"] = bench_legs.run(args.legs.split(","), hip, not args.no_cpu_baseline)
    elif rank_legs is not None:
        out["legs"] = rank_legs

    print(json.dumps(out), flush=True)
    barrier()


# newest committed PMC summary of this command (tools/profile.sh +
# tools/pmc_summary.py), per sweep launch
PMC_PROFILES = [os.path.join(ROOT, "profiles", "r06", "pmc.json"),
                os.path.join(ROOT, "profiles", "r05", "pmc.json"),
                os.path.join(ROOT, "profiles", "r04", "pmc.json"),
                os.path.join(ROOT, "profiles", "r03", "pmc.json"),
                os.path.join(ROOT, "profiles", "r02", "pmc.json"),
                os.path.join(ROOT, "profiles", "r01", "v6_pmc.json")]
PMC_PROFILE = next((p for p in PMC_PROFILES if os.path.exists(p)), PMC_PROFILES[-1])
SWEEP_KERNELS = ("spf_msbfs_kernel", "ms_finalize_kernel", "first_hop_lvl_kernel")


def pmc_traffic():
    """HBM bytes per sweep launch from the committed rocprofv3 PMC summary of
    this same command (tools/profile.sh + tools/pmc_summary.py: FETCH_SIZE
    doubled per the gfx950 wide-read correction, plus WRITE_SIZE), summed over
    the kernels of one sweep. PMC counters cannot be read from inside the
    timed run, so this is the profiled value, not a live one."""
    try:
        with open(PMC_PROFILE) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None, None
    total, seen = 0.0, []
    for name, k in prof.items():
        if any(s in name for s in SWEEP_KERNELS):
            if k.get("hbm_read_bytes") is None or k.get("hbm_write_bytes") is None:
                return None, None
            total += k["hbm_read_bytes"] + k["hbm_write_bytes"]
            seen.append(name.split("(")[0].replace("void ", ""))
    if len(seen) != len(SWEEP_KERNELS):
        return None, None
    return round(total), os.path.relpath(PMC_PROFILE, ROOT) + ": " + " + ".join(seen)


def profiled_build(solver_impl, me, als_impl, ps_impl):
    """One buildRouteDb with its phase times (the phases ORH_ROUTE_PROF
    prints), minor / major page faults and RSS growth across the call."""
    sec, n, phases, minflt, majflt, drss = solver_impl.time_build_route_db_phases(me, als_impl, ps_impl)
    return {"ms": sec * 1e3, "routes": n, "phases": phases, "minflt": minflt, "majflt": majflt,
            "rss_delta": drss}


def phase_summary(runs):
    """Per phase the median ms over the runs (a phase named twice in one build
    is summed), the phases' median total, and the median page faults / RSS
    growth per build."""
    names, per = [], []
    for r in runs:
        d = {}
        for name, ms in r["phases"]:
            name = name.strip()
            if name not in names:
                names.append(name)
            d[name] = d.get(name, 0.0) + ms
        per.append(d)
    med = {n: round(statistics.median(d.get(n, 0.0) for d in per), 3) for n in names}
    return {"phases_ms": med,
            "unaccounted_ms": round(statistics.median(
                r["ms"] - sum(ms for name, ms in r["phases"] if not name.strip().startswith("select:"))
                for r in runs), 3),
            "minor_faults": int(statistics.median(r["minflt"] for r in runs)),
            "major_faults": int(statistics.median(r["majflt"] for r in runs)),
            "rss_delta_mb": round(statistics.median(r["rss_delta"] for r in runs) / 2**20, 2)}


def cgroup_cpu_quota():
    """CPUs allowed by the cgroup v2 cpu.max quota (None: no quota)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        return None


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters (None where the file is absent)."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f if line.strip())}
    except (OSError, ValueError):
        return None


def throttle_delta(a, b):
    """CFS throttling between two cpu.stat snapshots: periods, throttled
    periods and throttled time (the quota's cost to the host pool)."""
    if not a or not b:
        return None
    return {"nr_periods": b.get("nr_periods", 0) - a.get("nr_periods", 0),
            "nr_throttled": b.get("nr_throttled", 0) - a.get("nr_throttled", 0),
            "throttled_ms": round((b.get("throttled_usec", 0) - a.get("throttled_usec", 0)) / 1e3, 3)}


def spread(xs):
    """median, min, max and (max - min) / median of repeated timings (ms)."""
    m = statistics.median(xs)
    return {"median": round(m, 3), "min": round(min(xs), 3), "max": round(max(xs), 3),
            "spread": round((max(xs) - min(xs)) / m, 3) if m else None, "ms": [round(x, 3) for x in xs]}


def usable_cpus():
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    return min(n, q) if q else n


def host_info():
    """CPU model and core counts of this host (BASELINE.md reporting rules)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": cgroup_cpu_quota(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(args, adj_dbs, prefixes, n, gpu_value):
    """Oracle (port of the reference LinkState::runSpf with its containers)
    on this host: a bounded, evenly spaced sample of the same 10k sources."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "build"))
    import importlib
    from openr_amd.facade import Backend, load_topology
    from openr_amd.types import K_TESTING_AREA
    oracle = Backend(importlib.import_module("openr_oracle"), "oracle")
    als, ps = load_topology(oracle, adj_dbs, prefixes)
    ls = als[K_TESTING_AREA]
    step = max(1, (n * n) // args.cpu_sample)
    sample = [str(i) for i in range(0, n * n, step)][:args.cpu_sample]
    sec1, _ = ls._impl.time_spf_sources(sample, 1)
    usable = usable_cpus()
    threads = max(1, min(args.cpu_threads or usable, usable))
    # >= cpu_sample sources and >= 2 per thread, evenly spaced over the grid
    k = max(args.cpu_sample, 2 * threads)
    sample_mt = [str((i * (n * n)) // k) for i in range(k)]
    secn, _ = ls._impl.time_spf_sources(sample_mt, threads)
    # the rate per thread count (how the 16 threads scale: allocator
    # contention vs box noise), on the same evenly spaced sample
    by_threads = {}
    for t in sorted({2, 4, 8, threads} - {1}):
        if t > threads:
            continue
        kt = max(args.cpu_sample, 2 * t)
        st, _ = ls._impl.time_spf_sources([str((i * (n * n)) // kt) for i in range(kt)], t)
        by_threads[t] = round(kt / st, 2)
    solver = oracle.spf_solver("1", True)
    db = adj_dbs[n * n // 2]
    flips = [0]

    def cold():  # same topology-changing update as the GPU measurement
        flips[0] ^= 1
        db.adjacencies[0].metric = 1 + flips[0]
        ls.update_adjacency_database(db)
        return solver._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3

    brdb = median_ms(cold, 3)
    db.adjacencies[0].metric = 1
    v1 = len(sample) / sec1
    vn = len(sample_mt) / secn
    return {
        "cpu_baseline": {"value": round(vn, 2), "unit": "SPF-sources/s", "cores": threads,
                         "kind": "port",
                         "sample": f"{len(sample_mt)} evenly spaced sources of the 10k grid, "
                                   f"runSpf on {threads} threads (every CPU this process may "
                                   f"use: affinity {len(os.sched_getaffinity(0))}, cgroup quota "
                                   f"{cgroup_cpu_quota()}), one deep LinkState copy per thread"},
        "cpu_baseline_per_core": round(vn / threads, 2),
        "cpu_baseline_by_threads": {"1": round(v1, 2), **{str(t): r for t, r in by_threads.items()},
                                    "note": "SPF-sources/s by oracle thread count, same box and sample"},
        "cpu_baseline_all_cores_linear": {
            "value": round(vn / threads * (os.cpu_count() or threads), 1),
            "cores": os.cpu_count(),
            "note": "per-core rate x nproc (linear extrapolation, not measured)"},
        "cpu_baseline_1t": {"value": round(v1, 2), "unit": "SPF-sources/s", "cores": 1,
                            "kind": "port", "sample": f"{len(sample)} sources"},
        "cpu_build_route_db_ms": round(brdb, 2),
        "cpu_host": host_info(),
        "speedup_vs_cpu": round(gpu_value / vn, 1),
    }


if __name__ == "__main__":
    main()
