"""Scheduler-extender front-end over the device mirror.

The reference scheduler calls an HTTP extender after its own filters and scores
(`core/generic_scheduler.go:497-525` findNodesThatPassExtenders, `:670-708` prioritizeNodes) through
`HTTPExtender` (`core/extender.go:273-438`): a JSON POST to `<urlPrefix>/<verb>` carrying
`ExtenderArgs`, answered with `ExtenderFilterResult`, `HostPriorityList` or
`ExtenderBindingResult` (`staging/src/k8s.io/kube-scheduler/extender/v1/types.go`).  This module
serves those verbs from the GPU engine, so a stock kube-scheduler can use the device path without
a rebuild: disable the in-tree filter/score plugins the device replaces, and list the extender
with `filterVerb: filter`, `prioritizeVerb: prioritize`, `bindVerb: bind`, `weight: 1`,
`nodeCacheCapable: true`.

  filter      one device cycle (kgpu_schedule_one, no assume) on the mirror synced with
              kgpu_apply_delta; the candidates that pass come back as NodeNames (or Nodes),
              every other candidate in FailedNodes with the failing plugin's reasons.
  prioritize  the same cycle's outcome per candidate.  mode "select" (default): 10 for the
              selectHost winner AMONG THE CANDIDATES the scheduler sent (the device's weighted
              totals of those nodes, the build's tie-break key), 0 otherwise -- the scheduler adds
              score * weight * (MaxNodeScore / MaxExtenderPriority) (generic_scheduler.go:703-707),
              so with no in-tree scorers its own selectHost lands on that node.  The scheduler may
              send a subset: numFeasibleNodesToFind already cut the list (generic_scheduler.go:436-441)
              and in-tree filters or earlier extenders may have trimmed it.  mode "total": the
              device's weighted score total of each node.
  bind        the pod is bound (optional `binder` callback) and its placement goes into the
              scheduler-cache mirror (AssumePod + FinishBinding, cache.go:338-381), so the next
              cycle sees it without an informer round trip.

A cycle is computed once per (pod UID, cache generation): filter and prioritize of one scheduling
cycle share it.  Calls are serialized (one engine, one stream).  The extender's own profile must
evaluate every node (percentageOfNodesToScore 100): the scheduler has already applied its cut to the
candidate list, and a second cut would drop valid candidates as "not evaluated".
"""
import collections
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np

from . import abi
from . import api
from . import tiebreak
from .compile import CompileError, Pools
from .framework import status_reasons

MAX_EXTENDER_PRIORITY = 10  # extender/v1/types.go:29
PENDING_MAX = 4096          # pods filtered but not (yet) bound that the extender remembers
PENDING_TTL = 600.0         # seconds: an unbound pod's record expires (unschedulable / bound elsewhere)


class ExtenderError(Exception):
    """Reported to the scheduler in the result's Error field."""


def _pod_uid(pod):
    return api.meta(pod).get("uid", "") or ""


class GpuExtender:
    def __init__(self, cache, mode="select", binder=None, clock=time.monotonic):
        """cache: a kgpu.cache.SchedulerCache holding the cluster (the extender's node cache:
        nodeCacheCapable).  binder(namespace, name, uid, node) -> error string or None, for the
        API-server binding itself (None: record the placement only)."""
        if mode not in ("select", "total"):
            raise ValueError("mode must be 'select' or 'total'")
        pct = getattr(cache.profile, "percentage_of_nodes_to_score", 100)
        if pct not in (None, 100):
            raise ValueError("the extender's profile must score every node (percentage_of_nodes_to_score 100): "
                             "the scheduler cuts the candidate list before calling the extender")
        self.cache = cache
        self.mode = mode
        self.binder = binder
        self.clock = clock
        self.lock = threading.Lock()
        self.seq = 0
        self._memo = None      # (uid, generation, cycle)
        # uid -> (pod, time) seen by filter / prioritize, awaiting bind; bounded (PENDING_MAX, oldest
        # first) and aged (PENDING_TTL): pods that never bind here must not accumulate
        self._pending = collections.OrderedDict()

    # ------------------------------------------------------------------ cycle
    def _cycle(self, pod):
        gen = self.cache.sync()
        uid = _pod_uid(pod)
        if self._memo and uid and self._memo[0] == uid and self._memo[1] == gen:
            return self._memo[2]
        pools = Pools()
        try:
            q = self.cache.compiler.compile_pod(pod, pools)
        except CompileError as e:
            raise ExtenderError(str(e))
        pc, _ = pools.finalize()
        seq = self.seq
        res, _ = self.cache.engine.schedule_one(np.array([q], abi.QUERY), pc, seq=seq, assume=False)
        self.seq += 1
        n = len(self.cache.list)
        words = self.cache.engine.filter_words(n)
        # the device's weighted total of every feasible node (framework.go:633-648): the candidates'
        # winner in select mode, the scores in total mode
        totals = np.zeros(n, np.int64)
        if self.cache.profile.scores:
            for name, w in self.cache.profile.scores:
                _, norm = self.cache.engine.scores(abi.SCORE_IDS[name], n)
                totals += norm * max(int(w), 1)
        else:
            totals[:] = 1  # no score plugins: every feasible node scores 1 (generic_scheduler.go:631-640)
        node = int(res["node"])
        cyc = {"words": words, "totals": totals, "winner": self.cache.list[node] if node >= 0 else None,
               "node": node, "error": node == -2, "seq": seq, "compiled": (q, pc),
               "n_scalars": int(q["scalars"]["count"]), "scalar_names": None, "reasons": {}}
        if uid:
            self._memo = (uid, gen, cyc)
            self._remember(uid, pod)
        return cyc

    def _remember(self, uid, pod):
        now = self.clock()
        self._pending.pop(uid, None)
        self._pending[uid] = (pod, now)
        while self._pending and (len(self._pending) > PENDING_MAX or
                                 now - next(iter(self._pending.values()))[1] > PENDING_TTL):
            self._pending.popitem(last=False)

    def _winner(self, cyc, names, idx):
        """selectHost over the candidates the device found feasible: the maximum of
        total << 40 | rank40 (the build's tie-break, kgpu/tiebreak.py).  When the candidates hold every
        node the device found feasible, that is the device's own selectHost pick."""
        feas = idx[cyc["words"][idx] == 0]
        if len(feas) == 0:
            return None
        if cyc["node"] >= 0 and len(np.unique(feas)) == int((cyc["words"] == 0).sum()):
            return cyc["winner"]
        prof = self.cache.profile
        keys = tiebreak.keys_np(cyc["totals"][feas], feas, int(getattr(prof, "seed", 0x7B)), cyc["seq"],
                                int(getattr(prof, "tie_break_mode", tiebreak.MODE_HASH)))
        return self.cache.list[int(feas[int(np.argmax(keys))])]

    def _reasons(self, cyc, pod, nm, i, w, filters):
        """The FailedNodes string of node nm (local index i, status word w).  Reasons depend on the word,
        the pod and -- for TaintToleration -- the node's taints, and for NodeResourcesFit's scalar
        resources on the node's columns: memoized per (word, taints) except in that last case."""
        plugin = filters[(w & 0xFF) - 1]
        memo = not (plugin == "NodeResourcesFit" and cyc["n_scalars"])
        if memo:
            taints = tuple((t.get("key", ""), t.get("value", ""), t.get("effect", ""))
                           for t in api.spec(self.cache.nodes.get(nm) or {}).get("taints") or []) \
                if plugin == "TaintToleration" else ()
            hit = cyc["reasons"].get((w, taints))
            if hit is not None:
                return hit
        if cyc["scalar_names"] is None:
            cyc["scalar_names"] = self.cache.compiler.scalar_names(pod)
        st = status_reasons(filters, self.cache.compiler, self.cache.nodes, pod, nm, w, handle=self.cache.engine.h,
                            node=i, compiled=cyc["compiled"], scalar_names=cyc["scalar_names"])
        out = ", ".join(st[2]) if st and st[2] else (st[1] if st else "")
        if memo:
            cyc["reasons"][(w, taints)] = out
        return out

    def _candidates(self, args):
        """ExtenderArgs -> (names, NodeList items or None, local node indices).  NodeNames when the
        scheduler treats the extender as node-cache capable, else the full Node objects
        (extender.go:293-304)."""
        names = args.get("NodeNames")
        items = None
        if names is None:
            nl = args.get("Nodes")
            if nl is None:
                raise ExtenderError("ExtenderArgs carries neither NodeNames nor Nodes")
            items = nl.get("items") or []
            names = [api.name_of(n) for n in items]
            self._sync_nodes(items)
        self.cache.sync()
        try:
            idx = self._indices(names)
        except KeyError as e:
            raise ExtenderError("node %r is not in the extender's node cache" % e.args[0])
        return names, items, idx

    def _indices(self, names):
        """The candidates' local node indices (numpy)."""
        ix = self.cache.index
        return np.fromiter((ix[nm] for nm in names), np.int64, len(names))

    def _sync_nodes(self, items):
        """Node objects sent with each call (nodeCacheCapable false) refresh the mirror's copy."""
        for n in items:
            old = self.cache.nodes.get(api.name_of(n))
            if old is None:
                self.cache.add_node(n)
            elif old != n:
                self.cache.update_node(old, n)

    # ------------------------------------------------------------------ verbs
    def filter(self, args):
        """ExtenderArgs -> ExtenderFilterResult (extender.go:273-338)."""
        try:
            with self.lock:
                pod = args.get("Pod") or {}
                names, items, idx = self._candidates(args)
                cyc = self._cycle(pod)
                if cyc["error"]:
                    raise ExtenderError("a score plugin failed for pod %s/%s" % (api.ns_of(pod), api.name_of(pod)))
                filters = [f for f in self.cache.profile.filters if f in abi.FILTER_IDS]
                w_all = cyc["words"][idx]
                keep = np.nonzero(w_all == 0)[0].tolist()
                failed = {}
                for k in np.nonzero(w_all != 0)[0].tolist():
                    nm, w = names[k], int(w_all[k])
                    if w == abi.STATUS_NOT_EVALUATED:
                        failed[nm] = "node not evaluated (percentageOfNodesToScore)"
                    else:
                        failed[nm] = self._reasons(cyc, pod, nm, int(idx[k]), w, filters)
        except ExtenderError as e:
            return {"Nodes": None, "NodeNames": None, "FailedNodes": None, "Error": str(e)}
        out = {"Nodes": None, "NodeNames": None, "FailedNodes": failed, "Error": ""}
        if items is None:
            out["NodeNames"] = [names[k] for k in keep]
        else:
            out["Nodes"] = {"metadata": {}, "items": [items[k] for k in keep]}
        return out

    def prioritize(self, args):
        """ExtenderArgs -> HostPriorityList (extender.go:340-382).  A failure is an HTTP error:
        the scheduler ignores a failing prioritizer (generic_scheduler.go:686-688)."""
        with self.lock:
            pod = args.get("Pod") or {}
            names, _, idx = self._candidates(args)
            cyc = self._cycle(pod)
            if self.mode == "select":
                winner = self._winner(cyc, names, idx)
                return [{"Host": nm, "Score": MAX_EXTENDER_PRIORITY if nm == winner else 0} for nm in names]
            sc = np.where(cyc["words"][idx] == 0, cyc["totals"][idx], 0).tolist()
            return [{"Host": nm, "Score": int(s)} for nm, s in zip(names, sc)]

    def bind(self, args):
        """ExtenderBindingArgs -> ExtenderBindingResult (extender.go:384-404)."""
        with self.lock:
            uid, node = args.get("PodUID", ""), args.get("Node", "")
            rec = self._pending.pop(uid, None)
            pod = rec[0] if rec is not None else None
            if pod is None:
                return {"Error": "pod %s/%s (uid %s) was not filtered by this extender" %
                                 (args.get("PodNamespace", ""), args.get("PodName", ""), uid)}
            if node not in self.cache.index:
                return {"Error": "node %r is not in the extender's node cache" % node}
            if self.binder is not None:
                err = self.binder(args.get("PodNamespace", ""), args.get("PodName", ""), uid, node)
                if err:
                    return {"Error": str(err)}
            placed = dict(pod)
            placed["spec"] = dict(api.spec(pod), nodeName=node)
            self.cache.assume_pod(placed)
            self.cache.finish_binding(placed, self.clock())
            self._memo = None
            return {"Error": ""}


# ---------------------------------------------------------------------- HTTP
class _Handler(BaseHTTPRequestHandler):
    ext = None
    prefix = ""

    def log_message(self, fmt, *a):  # quiet
        pass

    def do_POST(self):
        path = self.path
        if not path.startswith(self.prefix + "/"):
            return self._send(404, {"Error": "unknown path %s" % path})
        verb = path[len(self.prefix) + 1:]
        fn = {"filter": self.ext.filter, "prioritize": self.ext.prioritize, "bind": self.ext.bind}.get(verb)
        if fn is None:
            return self._send(404, {"Error": "unknown verb %s" % verb})
        try:
            n = int(self.headers.get("Content-Length", "0"))
            args = json.loads(self.rfile.read(n) or b"{}")
        except (ValueError, json.JSONDecodeError) as e:
            return self._send(400, {"Error": "bad request body: %s" % e})
        try:
            out = fn(args)
        except ExtenderError as e:      # prioritize: the scheduler treats non-200 as an error
            return self._send(500, {"Error": str(e)})
        self._send(200, out)

    def _send(self, code, obj):
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)


def serve(ext, host="127.0.0.1", port=0, prefix=""):
    """Start the extender's HTTP server in a daemon thread; returns (server, url prefix).
    The scheduler's `urlPrefix` is the returned URL."""
    handler = type("ExtHandler", (_Handler,), {"ext": ext, "prefix": prefix.rstrip("/")})
    srv = ThreadingHTTPServer((host, port), handler)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    return srv, "http://%s:%d%s" % (host, srv.server_address[1], prefix.rstrip("/"))
