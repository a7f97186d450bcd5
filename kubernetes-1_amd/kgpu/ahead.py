"""Batch-ahead: the throughput path (kgpu_schedule_batch, the persistent kernels) behind the per-pod
plugin boundary.

kube-scheduler runs one scheduling cycle per pod (scheduleOne, pkg/scheduler/scheduler.go:509-593);
a plugin sees one pod per PreFilter.  A cycle that starts with no batch in flight schedules the pod
TOGETHER WITH the pods the queue will pop next (the caller's `pending()`, in queue order:
PrioritySort, queuesort/priority_sort.go:41-50) in one kgpu_schedule_batch with on-device assume.
Pod k of the batch is evaluated with pods 0..k-1 assumed on their chosen nodes -- exactly the state
the per-pod cycle of pod k would see if nothing else happened in between.  The following cycles are
then served from the batch while that holds:

* the previous batch pod was assumed by the scheduler (cache.AssumePod, cache.go:338-361) on the node
  the batch chose: the device already holds it, so its UID is adopted (kgpu_adopt_pod) instead of
  sending an ADD_POD delta;
* nothing else changed in the cache (no other pod or node event since);
* the cycle's pod is the next pod of the batch, with the next sequence number.

Any deviation forgets the unconsumed speculative assumes (kgpu_forget_pod, newest first), syncs the
deviation like any other cycle, and starts a new batch.  Placements are therefore the per-pod
cycles' placements, pod for pod; only the work is batched.

This is the host mirror of go/gpueval/ahead.go (tests/test_ahead.py checks it against per-pod
cycles under queue-order changes, external events, failed binds and forgotten pods)."""
from collections import deque

import numpy as np

from . import abi
from .cache import _pod_key
from .compile import Pools


class _Entry:
    __slots__ = ("key", "seq", "host", "res", "slot")

    def __init__(self, key, seq, host, res, slot):
        self.key, self.seq, self.host, self.res, self.slot = key, seq, host, res, slot


class BatchAhead:
    def __init__(self, cache, pending, depth=256):
        """cache: a kgpu.cache.SchedulerCache; pending(): the pods the scheduling queue will pop next,
        in pop order (the current cycle's pod may or may not be among them)."""
        self.cache = cache
        self.pending = pending
        self.depth = max(1, int(depth))
        self.spec = deque()        # speculative results not yet handed out
        self.adopt = None          # the last handed-out placed entry, until its assume is seen
        self.stats = {"batches": 0, "batched_pods": 0, "served": 0, "invalidated": 0, "forgotten": 0}

    # ------------------------------------------------------------------ bookkeeping
    def _adopt_previous(self):
        """The previous cycle's pod: adopted when the cache's first change since is exactly its
        assume on the chosen node; otherwise it joins the entries to forget."""
        e, self.adopt = self.adopt, None
        if e is None:
            return
        log = self.cache._log
        if log and log[0][0] == "add" and log[0][1] == e.host and log[0][2] == e.key:
            self.cache.engine.adopt_pod(e.slot, self.cache.uid_ids.add(e.key))
            self.cache.dev_pods[e.key] = e.host
            del log[0]
        else:
            self.spec.appendleft(e)

    def _changed(self):
        c = self.cache
        return bool(c._log) or bool(c._dirty_nodes) or c._node_set_changed or c._lists_dirty

    def _invalidate(self):
        """Undo the speculative assumes still on the device, newest first (cache.ForgetPod)."""
        placed = [e for e in self.spec if e.host is not None]
        for e in reversed(placed):
            self.cache.engine.forget(e.slot)
        self.stats["forgotten"] += len(placed)
        self.stats["invalidated"] += 1
        self.spec.clear()

    # ------------------------------------------------------------------ one cycle
    def schedule(self, pod, seq):
        """One scheduling cycle (the GpuEval PreFilter): returns (host name or None, kgpu_result),
        as SchedulerCache.schedule does.  The caller assumes a placed pod through cache.assume_pod."""
        self._adopt_previous()
        key = _pod_key(pod)
        if self.spec:
            if not self._changed() and self.spec[0].key == key and self.spec[0].seq == seq:
                e = self.spec.popleft()
                if e.host is not None:
                    self.adopt = e
                self.stats["served"] += 1
                return e.host, e.res
            self._invalidate()
        return self._new_batch(pod, key, seq)

    def _new_batch(self, pod, key, seq):
        c = self.cache
        c.sync()
        pods = [pod]
        for p in self.pending():
            if len(pods) >= self.depth:
                break
            if _pod_key(p) != key:
                pods.append(p)
        pools = Pools()
        qs = []
        for p in pods:
            try:
                qs.append(c.compiler.compile_pod(p, pools))
            except Exception:  # a pod the compiler rejects ends the batch; its own cycle reports it
                if not qs:
                    raise
                break
        pods = pods[:len(qs)]
        pc, _ = pools.finalize()
        slot = c.engine.next_slot()
        res, _ = c.engine.schedule_batch(np.array(qs, abi.QUERY), pc, first_seq=seq)
        self.stats["batches"] += 1
        self.stats["batched_pods"] += len(pods)
        entries = []
        for k, p in enumerate(pods):
            node = int(res[k]["node"])
            host = c.list[node] if node >= 0 else None
            entries.append(_Entry(_pod_key(p), seq + k, host, res[k], slot if host is not None else -1))
            if host is not None:
                slot += 1
        first = entries[0]
        self.spec.extend(entries[1:])
        if first.host is not None:
            self.adopt = first
        return first.host, first.res

    def close(self):
        """Drop the speculation (forget every unadopted assume) -- before the cache is used without it."""
        self._adopt_previous()
        if self.spec:
            self._invalidate()
