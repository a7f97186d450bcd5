"""Host mirror of the scheduler cache, feeding the device mirror with kgpu_apply_delta.

The reference keeps NodeInfos in `schedulerCache` (pkg/scheduler/internal/cache/cache.go) and
copies the changed ones into the scheduling Snapshot at the start of every cycle (UpdateSnapshot,
cache.go:202-276).  This class mirrors that bookkeeping on the host -- nodes, the nodeTree,
podStates / assumedPods, NodeInfo pod sets (placeholder NodeInfos for pods whose node is unknown
included) -- and at `sync()` (UpdateSnapshot) sends the engine only what changed:

  * NodeInfo.AddPod / RemovePod of each pod event, by pod UID (KGPU_D_ADD_POD / REMOVE_POD);
  * NodeInfo.SetNode for added / updated nodes (KGPU_D_SET_NODE);
  * the Snapshot.List() rebuild (nodeTree.next() x numNodes, cache.go:278-301) when the node set
    changed, as a gather order executed on the device.

Anything the device columns cannot absorb (a new node label key, taint words or scalar resource)
falls back to a full kgpu_upload_snapshot of the mirror, in the mirror's own list order.
"""
import numpy as np

from . import abi
from . import api
from .compile import Compiler, NeedsUpload, Pools, StrDict
from .native import Engine


class CacheError(Exception):
    """An error the reference cache returns (or treats as fatal corruption)."""


def _pod_key(pod):
    """framework.GetPodKey (types.go:600-607): the pod UID."""
    uid = api.meta(pod).get("uid", "") or ""
    if uid == "":
        raise CacheError("Cannot get cache key for pod with empty UID")
    return uid


def _node_name(pod):
    return api.spec(pod).get("nodeName", "") or ""


class SchedulerCache:
    def __init__(self, profile, nodes=(), pods=(), cluster=None, device=0, ttl=30.0, pods_hint=(),
                 create_engine=True):
        self.profile = profile
        self.cluster = cluster
        self.device = device
        self.ttl = ttl
        self.tree = api.NodeTree()
        self.nodes = {}          # name -> v1.Node (cache.nodes entries that carry a Node)
        self.node_pods = {}      # name -> {uid: pod}: NodeInfo.Pods, placeholder NodeInfos included
        self.states = {}         # uid -> podState {"pod", "assumed", "deadline", "bound"}
        self.uid_ids = StrDict()
        self.pods_hint = list(pods_hint)
        self.generation = 0
        self.list = []           # device node order (Snapshot.List())
        self.index = {}
        self.dev_pods = {}       # uid -> node name: pods on device rows
        self._log = []           # NodeInfo ops since the last sync
        self._dirty_nodes = set()
        self._node_set_changed = False  # a node added or removed: UpdateSnapshot rebuilds the list
        self._lists_dirty = False       # some node's images / preferAvoidPods changed: resend the CSR
        self.engine = None
        self.compiler = None
        self.uploads = 0
        self.create_engine = create_engine
        for n in nodes:
            self.add_node(n)
        for p in pods:
            self.add_pod(p)
        self._upload()

    # ------------------------------------------------------------------ ids
    def uid(self, pod):
        return self.uid_ids.add(_pod_key(pod))

    # ------------------------------------------------------------------ NodeInfo ops
    def _add_pod(self, pod):
        """cache.addPod (cache.go:412-420): a placeholder NodeInfo when the node is unknown."""
        name = _node_name(pod)
        self.node_pods.setdefault(name, {})[_pod_key(pod)] = pod
        self._log.append(("add", name, _pod_key(pod), pod))

    def _remove_pod(self, pod):
        """cache.removePod (cache.go:437-450) -> NodeInfo.RemovePod (types.go:484-533)."""
        name = _node_name(pod)
        pods = self.node_pods.get(name)
        if pods is None:
            return
        key = _pod_key(pod)
        if key not in pods:
            raise CacheError("no corresponding pod %s in pods of node %s" % (api.name_of(pod), name))
        del pods[key]
        self._log.append(("remove", name, key, pod))

    def _update_pod(self, old, new):
        """cache.updatePod (cache.go:423-435)."""
        if _node_name(new) not in self.node_pods:
            return
        self._remove_pod(old)
        self._add_pod(new)

    # ------------------------------------------------------------------ pod events (cache.go:338-523)
    def assume_pod(self, pod):
        key = _pod_key(pod)
        if key in self.states:
            raise CacheError("pod %s is in the cache, so can't be assumed" % key)
        self._add_pod(pod)
        self.states[key] = {"pod": pod, "assumed": True, "deadline": None, "bound": False}

    def finish_binding(self, pod, now):
        st = self.states.get(_pod_key(pod))
        if st is not None and st["assumed"]:
            st["bound"] = True
            st["deadline"] = now + self.ttl

    def forget_pod(self, pod):
        key = _pod_key(pod)
        st = self.states.get(key)
        if st is not None and _node_name(st["pod"]) != _node_name(pod):
            raise CacheError("pod %s was assumed on %s but assigned to %s" % (key, _node_name(pod),
                                                                             _node_name(st["pod"])))
        if st is None or not st["assumed"]:
            raise CacheError("pod %s wasn't assumed so cannot be forgotten" % key)
        self._remove_pod(pod)
        del self.states[key]

    def add_pod(self, pod):
        key = _pod_key(pod)
        st = self.states.get(key)
        if st is not None and st["assumed"]:
            if _node_name(st["pod"]) != _node_name(pod):
                # added to a different node than it was assumed to: clean up (cache.go:470-477)
                try:
                    self._remove_pod(st["pod"])
                except CacheError:
                    pass
                self._add_pod(pod)
            st.update(assumed=False, deadline=None, pod=pod)
        elif st is None:
            self._add_pod(pod)
            self.states[key] = {"pod": pod, "assumed": False, "deadline": None, "bound": False}
        else:
            raise CacheError("pod %s was already in added state" % key)

    def update_pod(self, old, new):
        key = _pod_key(old)
        st = self.states.get(key)
        if st is None or st["assumed"]:
            raise CacheError("pod %s is not added to scheduler cache, so cannot be updated" % key)
        if _node_name(st["pod"]) != _node_name(new):
            raise CacheError("pod %s updated on a different node than previously added to" % key)
        self._update_pod(old, new)
        st["pod"] = new

    def remove_pod(self, pod):
        key = _pod_key(pod)
        st = self.states.get(key)
        if st is None or st["assumed"]:
            raise CacheError("pod %s is not found in scheduler cache, so cannot be removed from it" % key)
        if _node_name(st["pod"]) != _node_name(pod):
            raise CacheError("pod %s was assumed to be on %s but got added to %s" % (key, _node_name(pod),
                                                                                   _node_name(st["pod"])))
        self._remove_pod(st["pod"])
        del self.states[key]

    def cleanup_assumed(self, now):
        """cleanupAssumedPods (cache.go:704-737): expire bound assumed pods past their deadline."""
        for key in [k for k, st in self.states.items() if st["assumed"]]:
            st = self.states[key]
            if not st["bound"]:
                continue
            if now > st["deadline"]:
                self._remove_pod(st["pod"])
                del self.states[key]

    # ------------------------------------------------------------------ node events (cache.go:581-647)
    def add_node(self, node):
        name = api.name_of(node)
        self.node_pods.setdefault(name, {})
        if name not in self.nodes:
            self._node_set_changed = True
        self.nodes[name] = node
        self.tree.add_node(node)
        self._dirty_nodes.add(name)

    def update_node(self, old, new):
        name = api.name_of(new)
        if name not in self.node_pods:
            self.node_pods[name] = {}
            self.tree.add_node(new)
        if name not in self.nodes:
            self._node_set_changed = True
        prev = self.nodes.get(name)
        if prev is None or (prev.get("status") or {}).get("images") != (new.get("status") or {}).get("images") or \
                api.avoid_pods(prev) != api.avoid_pods(new):
            self._lists_dirty = True
        self.tree.update_node(old, new)
        self.nodes[name] = new
        self._dirty_nodes.add(name)

    def remove_node(self, node):
        name = api.name_of(node)
        if name not in self.node_pods:
            raise CacheError("node %s is not found" % name)
        # the NodeInfo goes with its pods (removeNodeInfoFromList); podStates keep them
        for key, pod in self.node_pods[name].items():
            self._log.append(("remove", name, key, pod))
        del self.node_pods[name]
        self.nodes.pop(name, None)
        self._node_set_changed = True
        if not self.tree.remove_node(node):
            raise CacheError("node %s in group %r was not found" % (name, api.zone_key(node)))
        self._dirty_nodes.discard(name)

    # ------------------------------------------------------------------ views
    def listed_pods(self):
        """Pods of the listed NodeInfos, in list order (what the Snapshot holds)."""
        out = []
        for nm in dict.fromkeys(self.list):
            out.extend(self.node_pods.get(nm, {}).values())
        return out

    def ordered_nodes(self):
        return [self.nodes[nm] for nm in self.list]

    # ------------------------------------------------------------------ device sync
    def _upload(self, names=None):
        """Full kgpu_upload_snapshot of the mirror (first sync, or a change deltas cannot carry).
        names: the list order this sync already took from the nodeTree (None: take it now)."""
        names = self.tree.list() if names is None else list(names)
        uniq = list(dict.fromkeys(names))
        ordered = [self.nodes[nm] for nm in uniq]
        existing = [p for nm in uniq for p in self.node_pods.get(nm, {}).values()]
        self.compiler = Compiler(self.profile, self.cluster)
        self.compiler.register(ordered, existing, self.pods_hint)
        snap, arrays, order = self.compiler.compile_snapshot(ordered, existing, ordered=ordered, uid_of=self.uid)
        self.config = self.compiler.config(self.device)
        self.generation += 1
        if self.create_engine:
            if self.engine is None:
                self.engine = Engine(self.config)
            self.engine.upload(snap, arrays, self.generation)
        self._snap = (snap, arrays)
        self.list = order
        self.index = {nm: i for i, nm in enumerate(order)}
        self.dev_pods = {_pod_key(p): _node_name(p) for p in existing}
        self._log.clear()
        self._dirty_nodes.clear()
        self._node_set_changed = False
        self._lists_dirty = False
        self.uploads += 1
        if len(uniq) != len(names):
            # a list holding one NodeInfo twice: upload it once, then alias it (kgpu_delta_batch.order)
            self._sync(True, names)

    def sync(self):
        """UpdateSnapshot: push the changes since the last sync.  Returns the generation."""
        old_list = self.list
        # updateAllLists after a node add / remove (cache.go:228-260): numNodes calls of
        # nodeTree.next() (cache.go:278-291), exactly once per sync.  The pass may list a NodeInfo
        # twice and skip another when the tree was mid-round (node_tree.go:147-170).
        reorder = self._node_set_changed
        new_list = self.tree.list() if reorder else old_list
        try:
            return self._sync(reorder, new_list)
        except NeedsUpload:
            self._upload(new_list)
            return self.generation

    def _sync(self, reorder, new_list):
        comp = self.compiler
        old_list, old_index = self.list, self.index
        if reorder:
            new_index = {}
            for i, nm in enumerate(new_list):
                new_index.setdefault(nm, i)  # a node's first row addresses all of its rows
            fresh = [nm for nm in new_index if nm not in old_index]
        else:
            new_index, fresh = old_index, []
        pools = Pools()
        rows, pods, deltas = [], [], []
        n_vals = [len(comp.nkeys.vals[k]) for k in range(comp.dims["K"])]
        n_zones0 = len(comp.zones)
        set_nodes = sorted({nm for nm in self._dirty_nodes if nm in new_index} | set(fresh), key=new_index.get)
        for nm in set_nodes:
            rows.append(comp.node_row(self.nodes[nm], pools))
            deltas.append((abi.D_SET_NODE, new_index[nm], 0, len(rows) - 1))
        dev = dict(self.dev_pods) if reorder else self.dev_pods  # copied: a NeedsUpload restarts from scratch
        if reorder:
            # pods of dropped nodes leave the device with their rows
            for uid, nm in list(dev.items()):
                if nm not in new_index:
                    del dev[uid]
        pod_items = {}

        def item(pod):
            k = id(pod)
            if k not in pod_items:
                pods.append(comp.compile_pod(pod, pools))
                pod_items[k] = len(pods) - 1
            return pod_items[k]

        fresh_set = set(fresh)
        for op, nm, key, pod in self._log:
            if nm not in new_index or nm in fresh_set:
                continue  # placeholder / dropped NodeInfo, or a node seeded below
            uid = self.uid_ids.add(key)
            if op == "add":
                deltas.append((abi.D_ADD_POD, new_index[nm], uid, item(pod)))
                dev[key] = nm
            else:
                deltas.append((abi.D_REMOVE_POD, new_index[nm], uid, item(pod)))
                dev.pop(key, None)
        for nm in fresh:
            for key, pod in self.node_pods.get(nm, {}).items():
                deltas.append((abi.D_ADD_POD, new_index[nm], self.uid_ids.add(key), item(pod)))
                dev[key] = nm
        if not deltas and not reorder:
            self._log.clear()
            self._dirty_nodes.clear()
            self._node_set_changed = False
            return self.generation
        batch = abi.DeltaBatch()
        keep = {}
        d = np.zeros(len(deltas), abi.DELTA)
        for i, (op, node, uid, it) in enumerate(deltas):
            d[i] = (op, node, uid, it, 0)
        keep["deltas"] = d
        keep["pods"] = np.array(pods, abi.QUERY) if pods else np.zeros(0, abi.QUERY)
        keep["rows"] = np.array(rows, abi.NODE_ROW) if rows else np.zeros(0, abi.NODE_ROW)
        batch.n_deltas, batch.deltas = len(d), abi.ptr(d)
        batch.n_pods, batch.pods = len(keep["pods"]), abi.ptr(keep["pods"])
        batch.n_rows, batch.rows = len(keep["rows"]), abi.ptr(keep["rows"])
        if reorder:
            row_of = {nm: r for r, nm in enumerate(set_nodes)}
            order = np.array([old_index[nm] if nm in old_index else -1 - row_of[nm] for nm in new_list], np.int32)
            keep["order"] = order
            batch.n_order, batch.order = len(order), abi.ptr(order)
        if [len(comp.nkeys.vals[k]) for k in range(comp.dims["K"])] != n_vals:
            km = comp.key_meta()
            keep.update(km)
            for f, a in km.items():
                setattr(batch, f, abi.ptr(a) if a.size else abi.ptr(np.zeros(1, a.dtype)))
                if not a.size:
                    keep[f + "_z"] = np.zeros(1, a.dtype)
                    setattr(batch, f, abi.ptr(keep[f + "_z"]))
        if reorder or self._lists_dirty:
            lists = comp.node_lists([self.nodes[nm] for nm in new_list], list(self.nodes.values()))
            keep.update(lists)
            for f, a in lists.items():
                if not a.size:
                    a = keep[f] = np.zeros(1, a.dtype)
                setattr(batch, f, abi.ptr(a))
        if len(comp.zones) != n_zones0:
            batch.n_zones = len(comp.zones)
        batch.pools, keep["_pools"] = pools.finalize()
        self.generation += 1
        if self.engine is not None:
            self.engine.apply_delta(batch, self.generation, len(d), keep)
        self.list, self.index = list(new_list), new_index
        if reorder:
            comp.set_order(new_list, first_wins=True)  # a node's first row addresses all of its rows
        self.dev_pods = dev
        self._log.clear()
        self._dirty_nodes.clear()
        self._node_set_changed = False
        self._lists_dirty = False
        self._last_batch = (batch, keep)
        return self.generation

    # ------------------------------------------------------------------ cycles
    def schedule(self, pod, seq=0):
        """One scheduling cycle on the synced mirror (no assume: the caller assumes through
        assume_pod, as scheduleOne does at Reserve).  Returns (host name or None, kgpu_result)."""
        self.sync()
        pools = Pools()
        q = self.compiler.compile_pod(pod, pools)
        pc, pnp = pools.finalize()
        res, _ = self.engine.schedule_one(np.array([q], abi.QUERY), pc, seq=seq, assume=False)
        node = int(res["node"])
        return (self.list[node] if node >= 0 else None), res

    def close(self):
        if self.engine is not None:
            self.engine.close()
            self.engine = None
