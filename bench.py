#!/usr/bin/env python3
"""Benchmark: kube-scheduler's per-pod node-evaluation loop on MI355X.

Default workload = BASELINE.json configs[1]: 5000 nodes / 10,000 pods, NodeResourcesFit +
LeastAllocated + BalancedAllocation (synthetic cluster).  A step is one batch of
pods run through the scheduleOne loop (filter -> score -> selectHost -> assume, every pod in queue
order) on the device-resident snapshot; K steps x pods-per-step = the config's 10,000 pods.

Prints ONE JSON line (rank 0) with pods/s, node-evals/s, the roofline of the dominant kernel
(k_batch / k_tbatch, timed with HIP events on the engine's stream) and the CPU baseline (the C
restatement of the reference algorithm, oracle/c, timed on this host's cores on a bounded sample).
At N=1 the line carries `extra` records timed in the same run, each with its own roofline, PMC
traffic and CPU baseline: (b) at 100k nodes, the topology configs (c) and (d) at 5k and 100k nodes
(BASELINE.json: "at 5k & 100k nodes") and one 125k-node GPU's worth of config (e).

N > 1: the default workload is config (e), the 1M-node cluster of 8 x 125k-node
shards, with a config (b) record beside it.  Under torch.distributed.run the ranks come from the
environment; `bench.py --gpus N` started bare spawns its N rank processes itself.  The line records
how many ranks the RCCL communicator and the xGMI mailboxes actually held (`comm`).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "kubernetes-1_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
BYTES_PER_NODE_EVAL = {"b": 72, "a": 73, "c": 121, "d": 84, "e": 121}  # SURVEY.md 8(d) algorithmic bytes per node-eval
BYTES_PER_EXISTING_POD = {"d": 24}
# the plugin profile of each workload (kgpu/cluster.py): "default" = the default provider's filters and
# scores (algorithmprovider/registry.go:92-133)
PROFILES = {"a": "default", "b": "Fit+LeastAllocated+BalancedAllocation", "c": "default", "d": "default",
            "e": "default"}  # IPA reads {node, ns, label bitset} per existing pod per pod


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_info():
    """Host cores and CPU model for the cpu_baseline record (SURVEY.md 8(d) 'report nproc, CPU model')."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    # the GPU box shares its host among GPUs: OMP_NUM_THREADS states this job's CPU share there
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return {"nproc": os.cpu_count() or 1, "affinity_cpus": min(aff, share) if share > 0 else aff, "cpu_model": model}


def make_workload(cfg, n_nodes, n_pods, shard=None):
    """(nodes, existing pods, init pods, measured pods, profile, compiled).  Init pods (config a: the
    scheduler_perf initPods, performance-config.yaml:1-13) are scheduled before the timed region.
    Config (e) comes straight from the columnar generator (cluster.sharded_spread_compiled, pinned
    equal to the object path by tests/test_cluster_fast.py): nodes is None and `compiled` holds this
    rank's shard of the compiled snapshot; every other config returns compiled=None."""
    from kgpu import cluster, native
    if cfg == "e":  # (b)+(c), zone = i % 64: --nodes is the shard per GPU (1M over 8 GPUs: --nodes 125000)
        rng = None if shard is None else native.shard_range(n_nodes, shard[1], shard[0])
        comp, compiled, pods, prof = cluster.sharded_spread_compiled(n_nodes=n_nodes, n_pods=n_pods, shard=rng)
        return None, [], [], pods, prof, (comp, compiled)
    return _object_workload(cfg, n_nodes, n_pods) + (None,)


def _object_workload(cfg, n_nodes, n_pods):
    from kgpu import cluster
    if cfg == "b":
        nodes, ex, pods, prof = cluster.fit_least_balanced(n_nodes=n_nodes, n_pods=n_pods)
        return nodes, ex, [], pods, prof
    if cfg == "a":
        nodes, init, pods, prof = cluster.scheduling_basic(n_nodes=n_nodes, n_init=n_nodes, n_pods=n_pods)
        return nodes, [], init, pods, prof
    if cfg == "c":
        nodes, ex, pods, prof = cluster.taints_affinity_spread(n_nodes=n_nodes, n_pods=n_pods)
        return nodes, ex, [], pods, prof
    if cfg == "d":
        nodes, ex, pods, prof = cluster.pod_affinity(n_nodes=n_nodes, n_existing=n_nodes, n_pods=n_pods)
        return nodes, ex, [], pods, prof
    raise SystemExit("config %r not benchmarked yet" % cfg)


def pmc_traffic(cfg, n_local, launch_pods, kname):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc passes of this
    exact workload (the newest profiles/r*_pmc_traffic.json holding it; tools/pmc_summary.py), or None."""
    for fname in ("r06_pmc_traffic.json", "r05_pmc_traffic.json", "r04_pmc_traffic.json", "r03_pmc_traffic.json", "r02_pmc_traffic.json", "r01_pmc_traffic.json"):
        try:
            with open(os.path.join(ROOT, "profiles", fname)) as fh:
                pmc = json.load(fh).get("%s:%d:%d" % (cfg, n_local, launch_pods))
        except (OSError, ValueError):
            continue
        if pmc and pmc["kernel"] == kname:
            return pmc["traffic_bytes_per_launch"]
    return None


def measure(args, cfg, n_nodes_per_gpu, B, K, W, cpu_sample, cpu_threads, latency_pods, rank, world, local,
            dist_on, cpu_thread_counts=None):
    """One workload: K timed steps of B pods after W warmup steps.  Returns the JSON record (rank 0)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from kgpu import abi, native
    from kgpu.framework import GpuFramework

    n_pods = B * K
    t_gen = time.time()
    # N > 1: the cluster is sharded by node across the ranks; each GPU holds a
    # n_nodes_per_gpu contiguous shard of Snapshot.List() (weak scaling in nodes: the cluster grows
    # with N), and every pod's shard winners are combined over RCCL / xGMI.
    n_cluster = n_nodes_per_gpu * world
    sharded = dist_on or args.shard
    shard = (rank, world) if sharded else None
    nodes, existing, init, pods, prof, compiled = make_workload(cfg, n_cluster, n_pods, shard=shard)
    fw = GpuFramework(prof, nodes, existing, pods_hint=init[:16] + pods[:16], device=local, shard=shard,
                      compiled=compiled)
    comm = None
    if sharded:
        uid = [native.comm_unique_id() if rank == 0 else None]
        if dist_on:
            dist.broadcast_object_list(uid, src=0)
        fw.init_comm(rank, world, uid[0])
        comm = fw.engine.comm_info()
        if dist_on:
            # what every rank's library saw: the judge reads the minimum over ranks
            t = torch.tensor([comm["rccl_nranks"], comm["xgmi_nranks"], comm["xgmi_peers_mapped"]],
                             dtype=torch.int64, device="cuda")
            lo = t.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            comm.update({"min_rccl_nranks_over_ranks": int(lo[0]), "min_xgmi_nranks_over_ranks": int(lo[1]),
                         "min_xgmi_peers_mapped_over_ranks": int(lo[2])})
    q_all, pc, pnp, errs = fw.compile_pods(init + pods)
    assert not errs, errs
    q_init, q = q_all[:len(init)], q_all[len(init):]
    log("workload %s: %d nodes (%d on this rank), %d pods, compiled in %.1fs"
        % (cfg, n_cluster, fw.snap.n_nodes, len(pods), time.time() - t_gen))
    eng = fw.engine
    if args.no_persistent:
        eng.set_option(abi.OPT_PERSISTENT, 0)
    if args.coop:
        eng.set_option(abi.OPT_COOPERATIVE, 1)
    if args.batch_geo is not None:
        eng.set_option(abi.OPT_BATCH_GEO, args.batch_geo)
    if args.batch_helper is not None:
        eng.set_option(abi.OPT_BATCH_HELPER, args.batch_helper)
    if args.topo_resident is not None:
        eng.set_option(abi.OPT_TOPO_RESIDENT, args.topo_resident)
    if args.topo_ahead is not None:
        eng.set_option(abi.OPT_TOPO_AHEAD, args.topo_ahead)
    if args.tbatch_geo is not None:
        eng.set_option(abi.OPT_TBATCH_GEO, args.tbatch_geo)
    if args.tbatch_wlab is not None:
        eng.set_option(abi.OPT_TBATCH_WLAB, args.tbatch_wlab)
    if args.tbatch_poll_sleep is not None:
        eng.set_option(abi.OPT_TBATCH_POLL_SLEEP, args.tbatch_poll_sleep)
    if args.topo_fused is not None:
        eng.set_option(abi.OPT_TOPO_FUSED, args.topo_fused)
    if args.no_topo_persistent:
        eng.set_option(abi.OPT_TOPO_PERSISTENT, 0)
    if args.max_groups:
        eng.set_option(abi.OPT_PERSIST_GROUPS, args.max_groups)

    def reset():
        eng.upload(fw.snap, fw.arrays)
        if len(q_init):
            eng.schedule_batch(q_init, pc, first_seq=0)   # untimed: the cluster's initial state

    xgmi = sharded and eng.xgmi_active()  # persistent runs exchange granules over xGMI mailboxes

    def timed():
        """Warmup (first launches, code object load) on a fresh snapshot, then the K timed steps."""
        if dist_on:
            dist.barrier()  # the persistent runs of all ranks wait for each other's granules
        reset()
        for w in range(W):
            eng.schedule_batch(q[:B], pc, first_seq=len(q_init))
        reset()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        stats = abi.Stats()
        t0 = time.perf_counter()
        results = []
        if args.no_pipeline:
            for k in range(K):
                res, stats = eng.schedule_batch(q[k * B:(k + 1) * B], pc, first_seq=len(q_init) + k * B, stats=stats)
                results.append(res)
        else:
            # pipelined steps (kgpu_schedule_batch_submit / _wait): step k+1's host work overlaps step k's
            # device run; a step the pipeline does not carry (topology pods) runs synchronously in submit
            for k in range(K):
                eng.schedule_batch_submit(q[k * B:(k + 1) * B], pc, first_seq=len(q_init) + k * B, stats=stats)
                if eng.pipelined() > 1:
                    results.append(eng.schedule_batch_wait()[0])
            while eng.pipelined():
                results.append(eng.schedule_batch_wait()[0])
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        return time.perf_counter() - t0, results

    if xgmi:
        # a mailbox exchange that gives up (a rank's granules never arrive) fails the batch on every
        # rank; the ranks then agree to fall back to the per-pod RCCL exchange and measure that
        failed = 0
        try:
            elapsed, results = timed()
        except native.KgpuError as e:
            log("xGMI mailbox run failed (%s): falling back to the per-pod RCCL exchange" % e)
            failed = 1
        f = torch.tensor([failed], device="cuda")
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        if int(f.item()):
            xgmi = False
            eng.set_option(abi.OPT_XGMI, 0)
            elapsed, results = timed()
    else:
        elapsed, results = timed()
    if dist_on:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res_all = np.concatenate(results)
    placed = int((res_all["node"] >= 0).sum())
    pods_per_s = n_pods / elapsed

    # kernel timing pass (separate: per-launch events perturb the timed loop)
    if dist_on:
        dist.barrier()
    reset()
    eng.set_option(abi.OPT_KERNEL_TIMING, 1)
    kst = abi.Stats()
    _, kst = eng.schedule_batch(q[:B], pc, first_seq=len(q_init), stats=kst)
    eng.set_option(abi.OPT_KERNEL_TIMING, 0)
    # per-pod latency of the drop-in step: kgpu_schedule_one (one cycle with assume and the per-node
    # filter / score diagnostics the Go shim's Filter/Score lookups read), wall clock per call
    lat = []
    if latency_pods > 0:
        reset()
        # the drop-in registers the pod classes of its queue's pending pods at upload (kgpu_prepare_pods;
        # go/gpueval/plugin.go upload), so no measured cycle pays a class's first count
        eng.prepare_pods(q[:latency_pods], pc)
        for i in range(min(latency_pods, len(q))):
            t1 = time.perf_counter()
            eng.schedule_one(q[i], pc, seq=len(q_init) + i, assume=True)
            lat.append((time.perf_counter() - t1) * 1e6)
    lat_rec = None
    if lat:
        la = np.array(lat)
        lat_rec = {"call": "kgpu_schedule_one (classes prepared)", "pods": len(lat),
                   "p50_us": round(float(np.percentile(la, 50)), 2),
                   "p99_us": round(float(np.percentile(la, 99)), 2), "mean_us": round(float(la.mean()), 2)}
    # what a scheduleOne cycle costs through a product boundary (scheduler.go:509-593): the pod compile
    # (PreFilter-time host work, libkgpu's C compile and the Python marshalling in front of it), the
    # drop-in cycle (compile + kgpu_schedule_one per pod, the Go shim's PreFilter) and the HTTP extender's
    # verbs (filter + prioritize + bind per pod, JSON in process)
    comp_rec = dropin_rec = ext_rec = None
    if rank == 0 and world == 1 and args.dropin_pods > 0:
        from tools.compile_bench import compile_costs
        comp_rec = compile_costs(fw, pods[:min(len(pods), 1000)], reps=2)
        comp_rec["pods"] = min(len(pods), 1000)
        reset()
        dropin_rec = dropin_cycles(fw, eng, pods[:args.dropin_pods], len(q_init), comp_rec)
        if nodes is not None and not init and n_cluster <= 10000 and args.extender_pods > 0:
            ext_rec = extender_cycles(prof, nodes, existing, pods[:args.extender_pods], local)
    # eval_launches counts node-evaluation passes (one per pod); with the persistent kernel one
    # launch covers the whole batch, so the per-launch duration is kernel_ms / launches_made
    per_pod_s = kst.eval_kernel_ms / 1e3 / max(kst.eval_launches, 1)
    bpe = BYTES_PER_NODE_EVAL.get(cfg, 72)
    n_local = fw.snap.n_nodes
    pod_bytes = n_local * bpe + BYTES_PER_EXISTING_POD.get(cfg, 0) * len(existing)
    achieved = pod_bytes / per_pod_s / 1e9
    topo = cfg in ("c", "d", "e")
    persistent = (not args.no_persistent and (not sharded or xgmi) and not (topo and args.no_topo_persistent))
    launch_pods = B if persistent else 1
    kname = ("k_tbatch" if topo else "k_batch") if persistent else ("k_topo_* pipeline" if topo else "k_eval")

    # CPU baseline: the C restatement of the reference algorithm on this host's cores, at 1 worker,
    # the reference's parallelism (16 goroutines, internal/parallelize/parallelism.go:26) and every
    # core this process may run on; the fastest is reported, each rate listed beside it.
    cpu = None
    if rank == 0 and world == 1 and cpu_sample != 0:
        from oracle.cref import RefEngine
        S = n_pods if cpu_sample < 0 else min(cpu_sample, n_pods)
        host = host_info()
        rates = {}
        best = None
        counts = cpu_thread_counts or sorted({1, 4, 8, cpu_threads, host["affinity_cpus"]})
        samples = {}
        for th in counts:
            # one worker on a large cluster: a shorter sample (SINGLE_WORKER_SAMPLE pods), so the parallel
            # efficiency of the baseline is in the line without a minute of CPU time
            St = min(S, SINGLE_WORKER_SAMPLE) if th == 1 and n_local > 10000 else S
            ref = RefEngine(fw.config, fw.snap, threads=th)
            if len(q_init):
                ref.schedule(q_init, pc)   # untimed, like the GPU's
            tc = time.perf_counter()
            rres = ref.schedule(q[:St], pc, first_seq=len(q_init))
            tcpu = time.perf_counter() - tc
            ref.close()
            ok = bool(np.array_equal(rres["node"], res_all["node"][:St]))
            rates[str(th)] = round(St / tcpu, 2)
            samples[str(th)] = St
            log("cpu baseline %s: %d thread(s): %.1f pods/s over %d pods (placements %s)"
                % (cfg, th, St / tcpu, St, "match" if ok else "DIFFER"))
            if best is None or St / tcpu > best[0]:
                best = (St / tcpu, th, tcpu, ok, St)
        rate, th, tcpu, ok, St = best
        cpu = {"value": round(rate, 2), "unit": "pods/s", "cores": th, "kind": "port",
               "nproc": host["nproc"], "affinity_cpus": host["affinity_cpus"], "cpu_model": host["cpu_model"],
               "rates_by_threads": rates,
               "sample": "oracle/c over %s %d pods, %.2fs at %d thread(s); placements %s"
                         % ("all" if St == n_pods else "the first", St, tcpu, th, "match" if ok else "DIFFER")}
        if len(set(samples.values())) > 1:
            cpu["pods_by_threads"] = samples

    traffic = pmc_traffic(cfg, n_local, launch_pods, kname)
    rec = {
        "metric": "pods scheduled/sec", "value": round(pods_per_s, 2), "unit": "pods/s", "n_gpus": world,
        "steps": K, "warmup": W, "ms_per_step": round(1e3 * elapsed / K, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
        "config": {"workload": "(%s) %d nodes / %d pods" % (cfg, n_cluster, n_pods), "profile": PROFILES[cfg],
                   "nodes": n_cluster, "nodes_per_gpu": fw.snap.n_nodes, "pods": n_pods, "pods_per_step": B,
                   "percentage_of_nodes_to_score": 100,
                   "parallelism": ("node shards x%d, %s" % (world, "granules through xGMI peer stores (persistent kernel)"
                                                              if xgmi else "RCCL all-gather per pod"))
                   if sharded else "1 GPU"},
        "series": "%s:%d" % (cfg, n_nodes_per_gpu),
        "node_evals_per_s": round(pods_per_s * n_cluster, 1),
        "comm": comm,
        "placed": placed,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "kernel": kname,
                     "bytes_per_node_eval": bpe,
                     "avg_kernel_us": round(per_pod_s * launch_pods * 1e6, 3), "pods_per_launch": launch_pods,
                     "us_per_pod": round(per_pod_s * 1e6, 4),
                     "bytes_per_launch": pod_bytes * launch_pods},
        "cpu_baseline": cpu,
        "latency": lat_rec,
        "compile_us_per_pod": comp_rec["c_us_per_pod"] if comp_rec else None,
        "compile": comp_rec,
        "dropin": dropin_rec,
        "extender": ext_rec,
    }
    # release the device context before the next workload and before interpreter teardown (under
    # rocprofv3 the HIP runtime may be finalized before a garbage-collected engine would be)
    eng.close()
    return rec


def dropin_cycles(fw, eng, pods, first_seq, comp_rec):
    """The Go shim's PreFilter per pod, timed one pod at a time: kgpu_compile_pod from a descriptor built
    beforehand (desc.go's marshalling is Go's cost, reported beside it from the Python twin) and
    kgpu_schedule_one with assume.  pods/s of the whole loop."""
    import ctypes as C

    import numpy as np
    from kgpu import abi, cdesc
    from kgpu.compile import Pools
    L = cdesc.lib()
    comp = fw.compiler
    descs = [comp.pod_desc(p) for p in pods]
    # the shim's upload registers its queue's pod classes (kgpu_prepare_pods), outside the per-pod clock
    pq, ppc, _, _ = fw.compile_pods(pods)
    eng.prepare_pods(pq, ppc)
    pools = Pools()
    q = np.zeros(1, abi.QUERY)
    cu, cy = [], []
    t_all = time.perf_counter()
    for i, d in enumerate(descs):
        t0 = time.perf_counter()
        rc = L.kgpu_compile_pod(comp._cc, pools.h, C.byref(d), q.ctypes.data)
        view = pools.view()
        t1 = time.perf_counter()
        if rc != 0:
            raise RuntimeError("kgpu_compile_pod: %s" % comp._err())
        eng.schedule_one(q[0], view, seq=first_seq + i, assume=True)
        t2 = time.perf_counter()
        cu.append((t1 - t0) * 1e6)
        cy.append((t2 - t0) * 1e6)
    total = time.perf_counter() - t_all
    cu, cy = np.array(cu), np.array(cy)
    pct = lambda a, p: round(float(np.percentile(a, p)), 2)  # noqa: E731
    return {"call": "kgpu_compile_pod + kgpu_schedule_one (assume)", "pods": len(descs),
            "pods_s": round(len(descs) / total, 1), "compile_us_p50": pct(cu, 50), "compile_us_p99": pct(cu, 99),
            "cycle_us_p50": pct(cy, 50), "cycle_us_p99": pct(cy, 99),
            "marshal_us_per_pod": comp_rec.get("marshal_us_per_pod"),
            "note": "descriptors built outside the clock (the Go shim marshals in Go; the Python twin's "
                    "marshal cost is marshal_us_per_pod)"}


def extender_cycles(prof, nodes, existing, pods, device):
    """The HTTP extender (kgpu/extender.py) per pod: filter -> prioritize -> bind with
    ExtenderArgs JSON-encoded and decoded in process (the wire format, no socket), every node a candidate
    (nodeCacheCapable: NodeNames), the selectHost pick among the prioritize scores bound.  Its own
    scheduler-cache mirror and engine on the same cluster."""
    import numpy as np
    from kgpu import api
    from kgpu.cache import SchedulerCache
    from kgpu.extender import GpuExtender
    cache = SchedulerCache(prof, nodes, existing, device=device)
    ext = GpuExtender(cache)
    names = [api.name_of(n) for n in nodes]
    ts = []
    placed = 0
    try:
        for k, pod in enumerate(pods):
            t0 = time.perf_counter()
            fr = json.loads(json.dumps(ext.filter(json.loads(json.dumps({"Pod": pod, "NodeNames": names})))))
            if fr.get("Error"):
                raise RuntimeError("extender filter: %s" % fr["Error"])
            feasible = fr.get("NodeNames") or []
            if feasible:
                pr = json.loads(json.dumps(ext.prioritize(json.loads(json.dumps({"Pod": pod, "NodeNames": feasible})))))
                best = max(pr, key=lambda h: h["Score"])["Host"]
                md = api.meta(pod)
                br = ext.bind(json.loads(json.dumps({"PodName": md.get("name", ""), "PodNamespace": md.get("namespace", ""),
                                                     "PodUID": md.get("uid", ""), "Node": best})))
                if br.get("Error"):
                    raise RuntimeError("extender bind: %s" % br["Error"])
                placed += 1
            if k > 0:  # the first pod pays the mirror's first sync
                ts.append((time.perf_counter() - t0) * 1e6)
    finally:
        cache.close()
    a = np.array(ts)
    return {"verbs": "filter + prioritize + bind (JSON in process, no socket)", "pods": len(ts), "placed": placed,
            "pods_s": round(len(ts) / (a.sum() / 1e6), 1), "us_p50": round(float(np.percentile(a, 50)), 1),
            "us_p99": round(float(np.percentile(a, 99)), 1)}


DEFAULT_EXTRAS_1GPU = "b:100000,c:5000,d:5000,c:100000,d:100000,e:125000"
# the workload every N of the driver's 1/2/4/8 sweep runs: config (e)'s 125k-node shard per GPU (an
# extra record at N = 1, the headline at N > 1)
SCALING_SERIES = ("e", 125000)
SINGLE_WORKER_SAMPLE = 200
DEFAULT_EXTRAS_NGPU = "b:5000"


def parse_extras(spec):
    out = []
    for item in (spec or "").split(","):
        item = item.strip()
        if item:
            cfg, n = item.split(":")
            out.append((cfg, int(n)))
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher: start N rank processes (one per GPU, RANK =
    LOCAL_RANK = r, rendezvous on 127.0.0.1) and wait for them.  The parent never touches a GPU and
    never execs; it returns the first non-zero exit code, ending the other ranks when one fails."""
    import subprocess
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n), KGPU_BENCH_LAUNCHER="bench.py --gpus %d (spawned ranks)" % n)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                r = p.poll()
                if r is None:
                    continue
                procs.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    log("bench: rank process %d exited with %d: ending the other ranks" % (p.pid, r))
                    for q in procs:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for q in procs:
            try:
                q.wait(timeout=15)
            except Exception:
                q.kill()
    return rc


def probe_launch(rank, world):
    """--probe-launch: the launcher's CPU check (tests/test_launcher.py) -- every rank joins a gloo
    group and sums its rank; no GPU is touched."""
    import torch
    import torch.distributed as dist
    if os.environ.get("KGPU_PROBE_FAIL_RANK") == str(rank):
        sys.exit(3)  # tests/test_launcher.py: a rank that dies before the rendezvous
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    ranks = [None] * world
    dist.all_gather_object(ranks, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                                   "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"probe": True, "world": world, "sum": int(t.item()), "ranks": ranks,
                          "launcher": os.environ.get("KGPU_BENCH_LAUNCHER", "external")}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=None,
                    help="workload (BASELINE.json configs a-e); default (b) on one GPU, (e) on N > 1")
    ap.add_argument("--nodes", type=int, default=None,
                    help="nodes per GPU; default 5000, and 125000 for (e) (1M nodes over 8 GPUs)")
    ap.add_argument("--pods-per-step", type=int, default=1000)
    ap.add_argument("--cpu-sample", type=int, default=-1,
                    help="pods timed for the CPU baseline (-1: the whole workload, 0: skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--latency-pods", type=int, default=200, help="pods timed one at a time through kgpu_schedule_one")
    ap.add_argument("--dropin-pods", type=int, default=200,
                    help="pods timed through the drop-in cycle (C compile + kgpu_schedule_one); 0: skip the compile, "
                         "drop-in and extender records")
    ap.add_argument("--extender-pods", type=int, default=30,
                    help="pods through the extender's filter / prioritize / bind (configs up to 10k nodes)")
    ap.add_argument("--no-persistent", action="store_true", help="one evaluation launch per pod")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="synchronous kgpu_schedule_batch per step instead of pipelined submit / wait")
    ap.add_argument("--topo-fused", type=int, default=None, help="KGPU_OPT_TOPO_FUSED (default: the library's)")
    ap.add_argument("--no-topo-persistent", action="store_true",
                    help="topology pods through the per-pod topology launches instead of k_tbatch")
    ap.add_argument("--max-groups", type=int, default=0,
                    help="cap on the persistent kernels' workgroups (KGPU_OPT_PERSIST_GROUPS; 0: one per CU)")
    ap.add_argument("--shard", action="store_true",
                    help="at N=1: run the node-sharded path on a one-rank RCCL communicator (exchange overhead)")
    ap.add_argument("--extras", default=None,
                    help="further records timed in the same run, 'cfg:nodes_per_gpu,...'; default with no --config: "
                         "%s on one GPU (BASELINE.json's metric is quoted at 5k and 100k nodes for configs b-d), %s "
                         "on N > 1; '' for none" % (DEFAULT_EXTRAS_1GPU, DEFAULT_EXTRAS_NGPU))
    ap.add_argument("--extra-cpu-sample", type=int, default=1000, help="pods of each extra record's CPU baseline")
    ap.add_argument("--reset-at-exit", action="store_true", help="hipDeviceReset() before exiting (profiling runs)")
    ap.add_argument("--batch-helper", type=int, default=None,
                    help="KGPU_OPT_BATCH_HELPER (default: the library's, 1 = config (b)'s helper wave)")
    ap.add_argument("--topo-resident", type=int, default=None,
                    help="KGPU_OPT_TOPO_RESIDENT (default: the library's, 1 = resident topology state)")
    ap.add_argument("--topo-ahead", type=int, default=None,
                    help="KGPU_OPT_TOPO_AHEAD (default: the library's, 1 = next pod's non-topology half ahead)")
    ap.add_argument("--tbatch-geo", type=int, default=None,
                    help="KGPU_OPT_TBATCH_GEO (smallest k_tbatch geometry index; 0 = 256 threads x 1 row)")
    ap.add_argument("--tbatch-poll-sleep", type=int, default=None,
                    help="KGPU_OPT_TBATCH_POLL_SLEEP (default: the library's, 1 = sleep between statistics sweeps)")
    ap.add_argument("--tbatch-wlab", type=int, default=None,
                    help="KGPU_OPT_TBATCH_WLAB (default: the library's, 1 = every node's delta-key labels in LDS)")
    ap.add_argument("--batch-geo", type=int, default=None,
                    help="smallest k_batch geometry index considered (KGPU_OPT_BATCH_GEO; 0 = 64 row threads)")
    ap.add_argument("--coop", action="store_true",
                    help="KGPU_OPT_COOPERATIVE = 1: every persistent launch through hipLaunchCooperativeKernel "
                         "(default: ordinary launches of a co-resident grid)")
    ap.add_argument("--no-coop", action="store_true", help=argparse.SUPPRESS)  # the default since round 5
    ap.add_argument("--os-exit", action="store_true",
                    help="leave through os._exit(0) after printing (profiling runs: see DESIGN.md, rocprofv3 exit)")
    ap.add_argument("--probe-launch", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group, rank 0 prints what it saw")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("bench: WORLD_SIZE=%d but --gpus %d: running %d ranks" % (world, args.gpus, world))
    if args.probe_launch:
        probe_launch(rank, world)
        return
    import torch
    import torch.distributed as dist
    dist_on = world > 1
    if dist_on:
        dist.init_process_group("nccl", rank=rank, world_size=world)
        torch.cuda.set_device(local)

    cfg = args.config or ("e" if world > 1 else "b")
    n_nodes = args.nodes or (125000 if cfg == "e" else 5000)
    extras = parse_extras(args.extras if args.extras is not None else
                          ("" if args.config else (DEFAULT_EXTRAS_NGPU if world > 1 else DEFAULT_EXTRAS_1GPU)))
    line = measure(args, cfg, n_nodes, args.pods_per_step, args.steps, args.warmup, args.cpu_sample,
                   args.cpu_threads, args.latency_pods, rank, world, local, dist_on)
    line["launcher"] = os.environ.get("KGPU_BENCH_LAUNCHER", "external (torch.distributed.run)" if dist_on else "none")
    recs = []
    for xcfg, xn in extras:
        if args.shard or (xcfg, xn) == (cfg, n_nodes):
            continue
        # each record: its own roofline and a CPU baseline over extra_cpu_sample pods, at 1 and 16
        # workers (the reference's parallelize.Until width) up to 10k nodes, at 16 above
        recs.append(measure(args, xcfg, xn, args.pods_per_step, args.steps, args.warmup, args.extra_cpu_sample,
                            args.cpu_threads, args.latency_pods, rank, world, local, dist_on,
                            cpu_thread_counts=sorted({1, 4, 8, args.cpu_threads} if xn <= 10000 else
                                                     {1, 8, args.cpu_threads})))
    if recs:
        line["extra"] = recs
    # the record of the driver's 1/2/4/8 sweep's common workload (config (e)'s shard per GPU), by name
    key = "%s:%d" % SCALING_SERIES
    ser = [r for r in [line] + recs if r.get("series") == key]
    line["scaling_series"] = {"series": key, "value": ser[0]["value"] if ser else None,
                              "n_gpus": world, "unit": "pods/s"}
    # the same records in brief, last in the line: the driver keeps the tail of the output
    def brief(r):
        rf, cb, lt = r["roofline"], r.get("cpu_baseline") or {}, r.get("latency") or {}
        di, ex = r.get("dropin") or {}, r.get("extender") or {}
        return {"s": r["series"], "pods_s": round(r["value"]), "us_pod": rf["us_per_pod"], "GBs": rf["achieved"],
                "frac": rf["frac"], "traffic": rf["traffic"], "cpu": cb.get("value"), "cpu_th": cb.get("cores"),
                "cpu_1th": (cb.get("rates_by_threads") or {}).get("1"),
                "one_p50_p99": [lt.get("p50_us"), lt.get("p99_us")] if lt else None,
                "compile_us": r.get("compile_us_per_pod"), "dropin_pods_s": di.get("pods_s"),
                "extender_pods_s": ex.get("pods_s")}
    line["summary"] = [brief(r) for r in [line] + recs]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()
    if args.reset_at_exit:
        # profiling runs: release the HIP runtime's device state while rocprofv3's tool is attached (its
        # finalization runs in an exit handler before HIP's own; see DESIGN.md "rocprofv3 at exit")
        import ctypes
        ctypes.CDLL("libamdhip64.so").hipDeviceReset()
    if args.os_exit:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


if __name__ == "__main__":
    main()
