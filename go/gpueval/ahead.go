package gpueval

// Batch-ahead: the throughput path (kgpu_schedule_batch, the persistent kernels) behind the per-pod
// PreFilter.  Host mirror: kubernetes-1_amd/kgpu/ahead.py, checked against per-pod cycles by
// tests/test_ahead.py.
//
// scheduleOne (pkg/scheduler/scheduler.go:509-593) runs one cycle per pod, and a plugin sees one pod
// per PreFilter.  A PreFilter that finds no batch in flight schedules its pod TOGETHER WITH the pods
// the queue will pop next -- the scheduler's unassigned pods from the shared informer, in the order of
// the default QueueSort (queuesort/priority_sort.go:41-50: priority, then the time the pod entered the
// queue, which track.go's queue clock follows) -- in one kgpu_schedule_batch with on-device assume.
// Pod k of the batch is evaluated with pods 0..k-1 assumed on their chosen nodes: exactly the state
// the per-pod cycle of pod k sees when nothing else happens in between.  The next PreFilters are
// served from the batch while that holds:
//
//   * the previous batch pod was reserved (Reserve, scheduler.go:586-593's assume) on the node the
//     batch chose: that node's NodeInfo differs from the mirror by exactly that pod, which the device
//     already holds -- the mirror takes it over and kgpu_adopt_pod registers its UID for the pod's
//     slot (no ADD_POD is sent);
//   * every other node the tracker marked still has the NodeInfo the mirror holds (a bind
//     confirmation, cache.AddPod of an assumed pod, marks the node without changing it);
//   * the cycle's pod is the next batch pod.
//
// Any deviation forgets the unconsumed speculative assumes (kgpu_forget_pod, newest first) and the
// cycle runs as a normal kgpu_schedule_one cycle.  Placements are the per-pod cycles' placements; only
// the work is batched.
//
// A batch-served cycle has no per-node status words: its Filter passes the chosen node only (the
// framework then takes it without scoring, generic_scheduler.go:184-191).  A pod the batch found
// unschedulable is re-run as a normal diagnostic cycle, so its FitError statuses (and preemption,
// which reads them) are the reference's.  Batch-ahead is off while pods are nominated (the
// two-pass filter runs one cycle at a time).

/*
#include "kgpu.h"
*/
import "C"

import (
	"sort"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/labels"
	"k8s.io/apimachinery/pkg/types"
	framework "k8s.io/kubernetes/pkg/scheduler/framework/v1alpha1"
)

type aheadEntry struct {
	uid  types.UID
	seq  int64
	res  C.kgpu_result
	slot int32 // pod-table slot of the speculative assume (-1: not placed)
	host string
	// the assume delta the device applied (kgpu_pod_query.req / .nz): adoption checks that the
	// scheduler's own NodeInfo.AddPod moved the node's sums by exactly this much
	req [3]int64
	nz  [2]int64
}

type ahead struct {
	depth int
	spec  []aheadEntry // handed out in order
	adopt *aheadEntry  // the last handed-out placed entry, until its Reserve is seen
}

func (e *engine) nextSlot() int32 { return int32(C.kgpu_next_slot(e.ctx)) }
func (e *engine) adoptPod(slot int32, uid int64) error {
	return kerr(e.ctx, C.kgpu_adopt_pod(e.ctx, C.int32_t(slot), C.int64_t(uid)))
}

func podPriority(p *v1.Pod) int32 {
	if p.Spec.Priority != nil {
		return *p.Spec.Priority
	}
	return 0
}

// pendingPods: the pods this profile's queue will pop next, in PrioritySort order.
func (g *GpuEval) pendingPods(self *v1.Pod, max int) []*v1.Pod {
	all, err := g.h.SharedInformerFactory().Core().V1().Pods().Lister().List(labels.Everything())
	if err != nil {
		return nil
	}
	out := make([]*v1.Pod, 0, 64)
	for _, p := range all {
		if p.Spec.NodeName != "" || p.UID == self.UID || p.DeletionTimestamp != nil ||
			p.Spec.SchedulerName != self.Spec.SchedulerName {
			continue
		}
		out = append(out, p)
	}
	at, bad := g.track.queueKeys(out)
	type ranked struct {
		p   *v1.Pod
		pri int32
		at  int64
	}
	rs := make([]ranked, 0, len(out))
	for i, p := range out {
		if !bad[i] { // waits in backoff / unschedulable: not popped next
			rs = append(rs, ranked{p, podPriority(p), at[i]})
		}
	}
	sort.SliceStable(rs, func(i, j int) bool {
		a, b := rs[i], rs[j]
		if a.pri != b.pri {
			return a.pri > b.pri
		}
		if (a.at < 0) != (b.at < 0) { // a pod the clock has not seen yet entered the queue last
			return a.at >= 0
		}
		if a.at != b.at {
			return a.at < b.at
		}
		return a.p.CreationTimestamp.Before(&b.p.CreationTimestamp)
	})
	out = out[:0]
	for _, r := range rs {
		out = append(out, r.p)
	}
	if len(out) > max {
		out = out[:max]
	}
	return out
}

// adoptPrevious: the last handed-out placed pod is taken over by the mirror when its node's NodeInfo
// now holds it (Reserve assumed it there); otherwise it joins the speculation to forget.  Returns
// false when the snapshot changed in any other way than that assume.
func (g *GpuEval) adoptPrevious(list []*framework.NodeInfo) (bool, error) {
	ah := g.ahead
	e := ah.adopt
	ah.adopt = nil
	marked := g.track.peek() // deltaFromSnapshot consumes the marks
	m := g.mir
	clean := len(list) == len(m.genAt)
	for _, nm := range marked {
		if e != nil && nm == e.host {
			continue
		}
		// a mark whose NodeInfo did not move (its event changed nothing, or has not reached the
		// cache: the snapshot this cycle sees is the mirror's either way) leaves the batch valid
		pos, ok := m.index[nm]
		if !clean || !ok || int(pos) >= len(list) || list[pos].Node() == nil ||
			list[pos].Node().Name != nm || list[pos].Generation != m.genAt[pos] {
			clean = false
		}
	}
	if e == nil {
		return clean, nil
	}
	pos, ok := m.index[e.host]
	if !ok || int(pos) >= len(list) {
		ah.spec = append([]aheadEntry{*e}, ah.spec...)
		return false, nil
	}
	ni := list[pos]
	old := m.pods[e.host]
	var assumed *v1.Pod
	same := len(ni.Pods) == len(old)+1
	for _, pi := range ni.Pods {
		if pi.Pod.UID == e.uid {
			assumed = pi.Pod
			continue
		}
		if op, ok := old[pi.Pod.UID]; !ok || op != pi.Pod {
			same = false
		}
	}
	// the device row is the mirror's last sums plus the assume delta it applied; the NodeInfo's sums
	// after cache.AssumePod (NodeInfo.AddPod, types.go:549-581: Requested with overhead CPU as
	// MilliValue, NonZeroRequested with the non-zero defaults) must equal them
	want := m.res[e.host]
	for k := 0; k < 3; k++ {
		want.req[k] += e.req[k]
	}
	for k := 0; k < 2; k++ {
		want.nz[k] += e.nz[k]
	}
	if assumed == nil || !same || m.nodes[e.host] != ni.Node() || resOf(ni) != want {
		// not (only) this pod's assume, or sums the device does not hold: the speculative assume is
		// undone and the node diffed
		ah.spec = append([]aheadEntry{*e}, ah.spec...)
		g.track.mark(e.host)
		return false, nil
	}
	if err := g.eng.adoptPod(e.slot, m.uid(e.uid)); err != nil {
		return false, err
	}
	cur := make(map[types.UID]*v1.Pod, len(ni.Pods))
	for _, pi := range ni.Pods {
		cur[pi.Pod.UID] = pi.Pod
	}
	m.pods[e.host] = cur
	m.gens[e.host] = ni.Generation
	m.res[e.host] = want
	m.genAt[pos] = ni.Generation
	m.slots[e.uid] = e.slot
	g.track.settle(e.host) // the mirror matches that NodeInfo again
	return clean, nil
}

// invalidate undoes the speculative assumes still on the device, newest first (cache.ForgetPod).
func (g *GpuEval) invalidate() error {
	ah := g.ahead
	for i := len(ah.spec) - 1; i >= 0; i-- {
		if ah.spec[i].slot >= 0 {
			if err := g.eng.forget(ah.spec[i].slot); err != nil {
				ah.spec = nil
				g.mir = nil // the engine invalidated its mirror: the next sync uploads
				return err
			}
		}
	}
	ah.spec = nil
	return nil
}

// serveAhead is PreFilter's batch-ahead step: (result, true) when the cycle is served from a batch.
// A miss leaves the mirror exactly as a per-pod cycle expects it (speculation undone).
func (g *GpuEval) serveAhead(pod *v1.Pod, seq int64) (C.kgpu_result, bool, error) {
	var zero C.kgpu_result
	list, err := g.h.SnapshotSharedLister().NodeInfos().List()
	if err != nil || g.mir == nil {
		return zero, false, err
	}
	clean, err := g.adoptPrevious(list)
	if err != nil {
		return zero, false, err
	}
	ah := g.ahead
	if len(ah.spec) > 0 && clean && !g.nominated && ah.spec[0].uid == pod.UID && ah.spec[0].seq == seq {
		e := ah.spec[0]
		ah.spec = ah.spec[1:]
		if e.slot >= 0 {
			ah.adopt = &e
		}
		return e.res, true, nil
	}
	if len(ah.spec) > 0 {
		if err := g.invalidate(); err != nil {
			return zero, false, err
		}
	}
	return zero, false, nil
}

// startBatch runs after this cycle's sync: the pod and the pods the queue pops next in one
// kgpu_schedule_batch with on-device assume.  Returns the pod's own result.
func (g *GpuEval) startBatch(pod *v1.Pod, q C.kgpu_pod_query, ps *poolSet, seq int64) (C.kgpu_result, bool, error) {
	var zero C.kgpu_result
	ah := g.ahead
	if g.nominated || ah.depth <= 1 {
		return zero, false, nil
	}
	pods := []*v1.Pod{pod}
	qs := []C.kgpu_pod_query{q}
	for _, np := range g.pendingPods(pod, ah.depth-1) {
		nq, err := g.comp.compilePod(np, g.defaultSelector(np), ps)
		if err != nil {
			break // that pod's own cycle reports it
		}
		pods = append(pods, np)
		qs = append(qs, nq)
	}
	if len(pods) == 1 {
		return zero, false, nil
	}
	var a arena
	defer a.free()
	slot := g.eng.nextSlot()
	res, err := g.eng.scheduleBatch(qs, ps.toC(&a), seq)
	if err != nil {
		g.mir = nil
		return zero, false, err
	}
	ah.spec = ah.spec[:0]
	var first aheadEntry
	for k := range pods {
		e := aheadEntry{uid: pods[k].UID, seq: seq + int64(k), res: res[k], slot: -1,
			req: [3]int64{int64(qs[k].req[0]), int64(qs[k].req[1]), int64(qs[k].req[2])},
			nz:  [2]int64{int64(qs[k].nz[0]), int64(qs[k].nz[1])}}
		if res[k].node >= 0 {
			e.slot = slot
			e.host = g.mir.names[res[k].node]
			slot++
		}
		if k == 0 {
			first = e
		} else {
			ah.spec = append(ah.spec, e)
		}
	}
	if first.slot >= 0 {
		ah.adopt = &first
	}
	return first.res, true, nil
}
