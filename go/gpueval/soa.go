package gpueval

// Device mirror of the scheduling Snapshot (mirror of kubernetes-1_amd/kgpu/cache.py sync; the
// records themselves come from libkgpu's compiler, compile.go):
//
//   * upload():   Snapshot.List() -> kgpu_snapshot SoA columns (node order = node index).
//   * sync():     at PreFilter, the Snapshot was just refreshed by cache.UpdateSnapshot
//                 (internal/cache/cache.go:202-301).  NodeInfo.Generation tells which NodeInfos
//                 changed; their pod sets are diffed by UID into KGPU_D_ADD_POD / REMOVE_POD,
//                 changed Node objects into KGPU_D_SET_NODE, and a changed list into the
//                 kgpu_delta_batch.order gather.  Anything the device columns cannot absorb
//                 (a new label key, more taint words, a new scalar resource) re-uploads.

/*
#include "kgpu.h"
#include "kgpu_compile.h"
*/
import "C"

import (
	"fmt"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/types"
	framework "k8s.io/kubernetes/pkg/scheduler/framework/v1alpha1"
)

var errNeedsUpload = fmt.Errorf("gpueval: change needs a full upload")

// mirror is what the device holds, per list position.
type mirror struct {
	names    []string
	index    map[string]int32            // first position of a node (aliases share it)
	gens     map[string]int64            // NodeInfo.Generation last sent
	nodes    map[string]*v1.Node         // Node object last sent
	pods     map[string]map[types.UID]*v1.Pod
	uids     map[types.UID]int64         // pod UID -> engine uid
	nextUID  int64
	gen      int64
	slots    map[types.UID]int32         // pod UID -> pod-table slot (kgpu_victim.slot)
	added    map[int]types.UID           // delta index -> UID of an ADD_POD in the pending batch
	genAt    []int64                     // NodeInfo.Generation last sent, by list position
	listData unsafe.Pointer              // backing array of the Snapshot.List() last synced
	labels   labelCounts                 // per key, nodes carrying each value (key_unique)
	res      map[string]nodeRes          // NodeInfo.Requested / NonZeroRequested last sent, by node name
}

// nodeRes: the resource sums of a NodeInfo the device row holds (NodeInfo.AddPod, types.go:549-581).
type nodeRes struct {
	req [3]int64 // Requested: MilliCPU, Memory, EphemeralStorage
	nz  [2]int64 // NonZeroRequested: MilliCPU, Memory
}

func resOf(ni *framework.NodeInfo) nodeRes {
	var r nodeRes
	if q := ni.Requested; q != nil {
		r.req = [3]int64{q.MilliCPU, q.Memory, q.EphemeralStorage}
	}
	if q := ni.NonZeroRequested; q != nil {
		r.nz = [2]int64{q.MilliCPU, q.Memory}
	}
	return r
}

// recordSlots keeps the pod-table slot of every pod the last delta batch added.
func (m *mirror) recordSlots(slots []int32) {
	for i, u := range m.added {
		if i < len(slots) && slots[i] >= 0 {
			m.slots[u] = slots[i]
		}
	}
	m.added = nil
}

func (m *mirror) uid(u types.UID) int64 {
	if id, ok := m.uids[u]; ok {
		return id
	}
	m.nextUID++
	m.uids[u] = m.nextUID
	return m.nextUID
}

// labelCounts: per node label key, how many listed nodes carry each value id; multi[k] counts the
// values carried by two or more nodes.  A key with multi 0 is hostname-like (kgpu_snapshot.key_unique,
// cluster-wide because this mirror sees the whole Snapshot).
type labelCounts struct {
	cnt   [][]int32
	multi []int32
}

func (lc *labelCounts) add(k, v int32, d int32) {
	for int(k) >= len(lc.cnt) {
		lc.cnt = append(lc.cnt, nil)
		lc.multi = append(lc.multi, 0)
	}
	for int(v) >= len(lc.cnt[k]) {
		lc.cnt[k] = append(lc.cnt[k], 0)
	}
	before := lc.cnt[k][v]
	lc.cnt[k][v] += d
	if before < 2 && lc.cnt[k][v] >= 2 {
		lc.multi[k]++
	} else if before >= 2 && lc.cnt[k][v] < 2 {
		lc.multi[k]--
	}
}

func (lc *labelCounts) unique(K int) []uint8 {
	out := make([]uint8, K)
	for k := 0; k < K; k++ {
		if k >= len(lc.multi) || lc.multi[k] == 0 {
			out[k] = 1
		}
	}
	return out
}

// deltaBuild accumulates one kgpu_delta_batch.
type deltaBuild struct {
	ps         *poolSet
	deltas     []C.kgpu_delta
	podsQ      []C.kgpu_pod_query
	rows       []C.kgpu_node_row
	rowOf      map[string]int
	labelMoved bool
}

// diffNode sends one NodeInfo's changes: SET_NODE when its Node object changed, then
// NodeInfo.RemovePod / AddPod (types.go:456-533) by UID for the pods gone, new or replaced.
func (g *GpuEval) diffNode(b *deltaBuild, ni *framework.NodeInfo, pos int32, wasListed bool) error {
	m, c := g.mir, g.comp
	nm := ni.Node().Name
	if !wasListed || m.nodes[nm] != ni.Node() {
		if _, done := b.rowOf[nm]; !done {
			r, err := c.nodeRow(ni.Node(), b.ps)
			if err != nil {
				return err
			}
			b.rows = append(b.rows, r)
			b.rowOf[nm] = len(b.rows) - 1
			b.deltas = append(b.deltas, C.kgpu_delta{op: C.KGPU_D_SET_NODE, node: C.int32_t(pos), item: C.int32_t(len(b.rows) - 1)})
			if old := m.nodes[nm]; old != nil {
				for _, kv := range c.nodeLabelIDs(old) {
					m.labels.add(kv[0], kv[1], -1)
				}
			}
			for _, kv := range c.nodeLabelIDs(ni.Node()) {
				m.labels.add(kv[0], kv[1], 1)
			}
			b.labelMoved = true
		}
	}
	podDelta := func(pod *v1.Pod, op C.int32_t) error {
		q, err := c.compilePod(pod, nil, b.ps) // NodeInfo.AddPod / RemovePod read no DefaultSelector
		if err != nil {
			return err
		}
		b.podsQ = append(b.podsQ, q)
		if op == C.KGPU_D_ADD_POD {
			if m.added == nil {
				m.added = map[int]types.UID{}
			}
			m.added[len(b.deltas)] = pod.UID
		}
		b.deltas = append(b.deltas, C.kgpu_delta{op: op, node: C.int32_t(pos), uid: C.int64_t(m.uid(pod.UID)),
			item: C.int32_t(len(b.podsQ) - 1)})
		return nil
	}
	old := m.pods[nm]
	cur := make(map[types.UID]*v1.Pod, len(ni.Pods))
	for _, pi := range ni.Pods {
		cur[pi.Pod.UID] = pi.Pod
	}
	if wasListed {
		for u, pod := range old { // NodeInfo.RemovePod of pods gone or changed
			if np, ok := cur[u]; !ok || np != pod {
				if err := podDelta(pod, C.KGPU_D_REMOVE_POD); err != nil {
					return err
				}
			}
		}
	}
	for u, pod := range cur { // NodeInfo.AddPod of new or changed pods
		if op, ok := old[u]; wasListed && ok && op == pod {
			continue
		}
		if err := podDelta(pod, C.KGPU_D_ADD_POD); err != nil {
			return err
		}
	}
	m.pods[nm] = cur
	m.gens[nm] = ni.Generation
	m.nodes[nm] = ni.Node()
	m.res[nm] = resOf(ni)
	return nil
}

// deltaFromSnapshot diffs the refreshed Snapshot against the mirror.  Returns the C batch (in the
// arena) or errNeedsUpload.
//
// Cost.  UpdateSnapshot rebuilds Snapshot.List() only when a node was added or removed
// (cache.go:258-301); otherwise the list is the same slice and its NodeInfos are updated in place
// (cache.go:236-243: `*existing = *clone`).  So an unchanged list is recognized in O(1) (same backing
// array, same length), and only the NodeInfos the tracker marked (track.go: Reserve / Unreserve and the
// informers' pod and node events) are compared by generation: O(changed), as UpdateSnapshot's own walk
// of the cache's generation-ordered list.  Every fullEvery syncs (and with ExactSync, every sync) all
// positions' generations are compared as well, a tight loop over a slice.  A rebuilt list takes the
// full walk (node adds / removes are rare).
func (g *GpuEval) deltaFromSnapshot(list []*framework.NodeInfo, a *arena) (*C.kgpu_delta_batch, error) {
	m, c := g.mir, g.comp
	ps, err := newPoolSet()
	if err != nil {
		return nil, err
	}
	a.onFree(ps.free) // the batch's queries and rows point into it until kgpu_apply_delta returns
	b := &deltaBuild{ps: ps, rowOf: map[string]int{}}
	g.syncs++
	same := len(list) == len(m.names) && (len(list) == 0 || unsafe.Pointer(&list[0]) == m.listData)
	var order []int32
	if same {
		if g.exact || g.syncs%fullEvery == 0 || g.track.takeFull() {
			for i, ni := range list {
				if int32(i) != m.index[ni.Node().Name] || ni.Generation == m.genAt[i] {
					continue // an alias position, or unchanged
				}
				if err := g.diffNode(b, ni, int32(i), true); err != nil {
					return nil, err
				}
				m.genAt[i] = ni.Generation
				g.track.settle(ni.Node().Name)
			}
		} else {
			for _, nm := range g.track.take() {
				i, ok := m.index[nm]
				if !ok {
					continue // not listed: its add shows as a rebuilt list
				}
				ni := list[i]
				if ni.Generation == m.genAt[i] {
					continue // the event has not reached the cache yet: the mark stays (markTTL)
				}
				if err := g.diffNode(b, ni, i, true); err != nil {
					return nil, err
				}
				m.genAt[i] = ni.Generation
				g.track.settle(nm)
			}
		}
	} else {
		// the list was rebuilt: new positions, every NodeInfo compared
		names := make([]string, len(list))
		newIndex := make(map[string]int32, len(list))
		for i, ni := range list {
			names[i] = ni.Node().Name
			if _, ok := newIndex[names[i]]; !ok {
				newIndex[names[i]] = int32(i)
			}
		}
		order = make([]int32, len(names))
		for _, ni := range list {
			nm := ni.Node().Name
			if _, known := m.index[nm]; !known {
				if err := g.diffNode(b, ni, newIndex[nm], false); err != nil {
					return nil, err
				}
			}
		}
		for i, nm := range names {
			if j, ok := m.index[nm]; ok {
				order[i] = j
			} else {
				order[i] = int32(-1 - b.rowOf[nm])
			}
		}
		for _, ni := range list {
			nm := ni.Node().Name
			if _, known := m.index[nm]; known && (m.gens[nm] != ni.Generation || m.nodes[nm] != ni.Node()) {
				if err := g.diffNode(b, ni, newIndex[nm], true); err != nil {
					return nil, err
				}
			}
		}
		// labels of the nodes that left the list
		for nm, n := range m.nodes {
			if _, ok := newIndex[nm]; !ok {
				for _, kv := range c.nodeLabelIDs(n) {
					m.labels.add(kv[0], kv[1], -1)
				}
				delete(m.nodes, nm)
				delete(m.pods, nm)
				delete(m.gens, nm)
				delete(m.res, nm)
				b.labelMoved = true
			}
		}
		m.names, m.index = names, newIndex
		m.genAt = make([]int64, len(list))
		for i, ni := range list {
			m.genAt[i] = ni.Generation
		}
		if len(list) > 0 {
			m.listData = unsafe.Pointer(&list[0])
		}
	}
	bt := (*C.kgpu_delta_batch)(a.alloc(int(unsafe.Sizeof(C.kgpu_delta_batch{}))))
	bt.n_deltas, bt.deltas = C.int32_t(len(b.deltas)), cDeltas(a, b.deltas)
	bt.n_pods, bt.pods = C.int32_t(len(b.podsQ)), cQueries(a, b.podsQ)
	bt.n_rows, bt.rows = C.int32_t(len(b.rows)), cNodeRows(a, b.rows)
	if !same {
		bt.n_order, bt.order = C.int32_t(len(order)), ci32(a, order)
	}
	if !same || len(b.rows) > 0 {
		nodes := make([]*v1.Node, len(list))
		for i, ni := range list {
			nodes[i] = ni.Node()
		}
		// ImageLocality / NodePreferAvoidPods CSR over the new list; label dictionaries may have grown
		if err := c.nodeLists(nodes, bt, a); err != nil {
			return nil, err
		}
		if err := c.keyMeta(bt, a); err != nil {
			return nil, err
		}
	}
	if b.labelMoved {
		bt.key_unique = cu8(a, m.labels.unique(c.dims.K))
	}
	bt.n_zones = C.int32_t(c.dictSize(C.KGPU_DICT_ZONE, 0))
	bt.pools = *ps.toC(a)
	if !same {
		// node names (NodeName, matchFields) resolve against the new list from the next compile on
		if err := c.setOrder(m.names); err != nil {
			return nil, err
		}
	}
	return bt, nil
}
