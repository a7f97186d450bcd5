"""Batch-ahead (kgpu/ahead.py): the throughput path behind the per-pod boundary must give the
per-pod cycles' placements, pod for pod.

Two scheduler-cache mirrors (kgpu/cache.py) start from the same cluster and receive the same
events.  One schedules every pod with its own cycle (SchedulerCache.schedule: UpdateSnapshot +
kgpu_schedule_one); the other through BatchAhead (one kgpu_schedule_batch with on-device assume for
the pods the queue pops next, then adoption of each assume).  The scheduler loop pops pods in queue
order and assumes each placed pod on its host (cache.AssumePod).  Deviations the batch must survive
exactly: an external pod added and a node updated mid-stream, bind confirmations of assumed pods
arriving two cycles late (the cache's AddPod of an assumed pod changes nothing), a placed pod the scheduler does not
assume (a failed Reserve / Permit), a pod that jumps the queue, a pod deleted from the queue, and a
batch pod that turns out unschedulable.  After the stream, every node row of both devices must be
equal, and equal to the C restatement's rows of the final cluster."""
import copy

import numpy as np
import pytest

from kgpu import cluster
from kgpu.ahead import BatchAhead
from kgpu.cache import SchedulerCache

COLS = ("req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "num_pods")


def _workload(name):
    if name == "b":
        nodes, existing, pods, prof = cluster.fit_least_balanced(n_nodes=300, n_pods=400)
    elif name == "c":
        nodes, existing, pods, prof = cluster.taints_affinity_spread(n_nodes=240, n_pods=260)
    else:
        nodes, existing, pods, prof = cluster.pod_affinity(n_nodes=160, n_existing=160, n_pods=220)
    for i, p in enumerate(pods):
        p["metadata"]["uid"] = "q%d" % i
    return nodes, existing, pods, prof


def _run(name, batched, depth=64):
    nodes, existing, pods, prof = _workload(name)
    cache = SchedulerCache(prof, nodes, existing, pods_hint=pods[:32])
    queue = list(pods)
    big = copy.deepcopy(pods[5])
    big["metadata"].update(uid="huge", name="huge")
    big["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "100000", "memory": "1Ti"}}
    queue.insert(37, big)                       # unschedulable in the middle of a batch
    jumper = copy.deepcopy(pods[3])
    jumper["metadata"].update(uid="jumper", name="jumper")
    ahead = BatchAhead(cache, lambda: [p for p in queue if p["metadata"]["uid"] != "jumper"], depth=depth) \
        if batched else None
    hosts = []
    seq = 0
    step = 0
    unconfirmed = []
    while queue:
        if step == 90:
            queue.insert(0, jumper)             # pops before the pods the batch predicted
        if step == 120:
            queue.pop(3)                        # a predicted pod leaves the queue
        pod = queue.pop(0)
        if ahead is not None:
            host, _ = ahead.schedule(pod, seq)
        else:
            host, _ = cache.schedule(pod, seq=seq)
        seq += 1
        hosts.append((pod["metadata"]["uid"], host))
        if host is not None and step != 60:     # step 60: placed, but the scheduler does not assume it
            placed = copy.deepcopy(pod)
            placed["spec"]["nodeName"] = host
            cache.assume_pod(placed)
            unconfirmed.append(placed)
        if len(unconfirmed) > 2:                # the informer confirms the bind of an older assume
            cache.add_pod(unconfirmed.pop(0))   # (cache.go:466-481): no change, the batch survives
        if step == 150:                         # an external pod lands on a node
            ext = copy.deepcopy(pods[0])
            ext["metadata"].update(uid="ext", name="ext")
            ext["spec"]["nodeName"] = cache.list[7]
            cache.add_pod(ext)
        if step == 180:                         # a node's allocatable changes
            nm = cache.list[11]
            old = cache.nodes[nm]
            new = copy.deepcopy(old)
            new["status"]["allocatable"]["cpu"] = "2"
            cache.update_node(old, new)
        step += 1
    stats = dict(ahead.stats) if ahead is not None else None
    if ahead is not None:
        ahead.close()
    cache.sync()
    rows = cache.engine.read_nodes(len(cache.list))
    lst = list(cache.list)
    cache.close()
    return hosts, rows, lst, stats


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["b", "c", "d"])
def test_batch_ahead_equals_per_pod_cycles(name):
    want, rows_w, list_w, _ = _run(name, batched=False)
    got, rows_g, list_g, stats = _run(name, batched=True)
    assert list_g == list_w
    assert len(got) == len(want)
    for k, (a, b) in enumerate(zip(got, want)):
        assert a == b, (name, k, a, b)
    assert sum(1 for _, h in want if h is None) >= 1        # the unschedulable pod took part
    for c in COLS:
        np.testing.assert_array_equal(rows_g[c], rows_w[c], err_msg=c)
    # most cycles were served from batches; every deviation cost one new batch
    assert stats["served"] > len(got) // 2, stats
    assert stats["invalidated"] >= 3, stats
