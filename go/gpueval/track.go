package gpueval

// Change tracking for the device mirror: which NodeInfos of the Snapshot may have moved since the
// last sync, so that PreFilter's sync is O(changed) instead of a walk of Snapshot.List().
//
// The reference's UpdateSnapshot (internal/cache/cache.go:218-247) walks the cache's
// generation-ordered node list from its head and stops at the first NodeInfo not newer than the
// snapshot.  A plugin sees only the Snapshot (FrameworkHandle.SnapshotSharedLister), not that list, so
// it learns of changes from the same sources the cache does:
//
//   * Reserve / Unreserve (interface.go:332-368): the node of every assume / forget the scheduler
//     makes (scheduler.go:586-593 assume, the binding cycle's ForgetPod);
//   * the shared informers' pod and node events (eventhandlers.go:93-295 feed the cache from the same
//     informers): a pod's old and new nodeName, a node's name.
//
// A marked node is re-checked at every sync until its NodeInfo.Generation moves (an event can reach
// this handler before the cache applied it) or markTTL syncs passed.  A mark that expires without
// its generation moving forces a full generation scan at the next sync: the cache may simply be
// later than markTTL syncs in applying the event (informer listeners run on their own goroutines),
// and the scan then finds the change whenever it lands.  Nothing can reach the cache without passing
// through one of these sources except an assumed pod's expiry (cache.cleanupAssumedPods,
// cache.go:704-737) and an event whose handler ran late, so every fullEvery syncs the whole list's
// generations are compared as well (a tight loop over positions: no map operations).  ExactSync in
// the plugin args compares every generation at every sync.
//
// Nominations.  The same pod events record every node named by an unassigned pod's
// Status.NominatedNodeName, and SelectNodesForPreemption records its candidate nodes (the one the
// scheduler nominates is among them, before the status update reaches the informer).  PreFilter asks
// the PodNominator only about those nodes and the ones that held nominated pods at the last sync:
// O(nominated) instead of NominatedPodsForNode on every listed node (preempt.go syncNominated).
//
// Queue clock (batch-ahead's prediction of the pods the queue pops next, ahead.go pendingPods).
// PrioritySort orders by priority, then QueuedPodInfo.Timestamp: set when the pod enters the queue
// (scheduling_queue.go:248 Add, :458 Update of a pod in no queue, both through newQueuedPodInfo
// :632) and reset when a cycle fails (AddUnschedulableIfNotPresent, :306); updates and moves between
// the sub-queues keep it (updatePod :657).  The same informer events stamp a logical tick on every
// unassigned pod; a cycle that did not reach Reserve, or an Unreserve, re-stamps its pod and marks it
// failed: a failed pod waits in the backoff or unschedulable queue, so it is left out of the
// prediction until its next cycle starts.

import (
	"sync"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/types"
	"k8s.io/client-go/tools/cache"
)

const (
	markTTL   = 32   // syncs a mark stays without its NodeInfo's generation moving
	fullEvery = 1024 // syncs between full generation scans
)

type tracker struct {
	mu    sync.Mutex
	marks map[string]int // node name -> syncs left
	full  bool           // a mark expired unsettled: compare every generation at the next sync
	noms  map[string]struct{}

	tick   int64                  // queue clock
	queued map[types.UID]int64    // unassigned pod -> tick it entered the queue (Timestamp)
	failed map[types.UID]struct{} // its last cycle failed: in backoff / unschedulable
}

func newTracker() *tracker {
	return &tracker{marks: map[string]int{}, noms: map[string]struct{}{},
		queued: map[types.UID]int64{}, failed: map[types.UID]struct{}{}}
}

// enqueue stamps a pod entering the queue; a pod already queued keeps its stamp (updatePod).
func (t *tracker) enqueue(uid types.UID) {
	t.mu.Lock()
	if _, ok := t.queued[uid]; !ok {
		t.queued[uid] = t.tick
		t.tick++
	}
	t.mu.Unlock()
}

// dequeue forgets a pod that was bound or deleted.
func (t *tracker) dequeue(uid types.UID) {
	t.mu.Lock()
	delete(t.queued, uid)
	delete(t.failed, uid)
	t.mu.Unlock()
}

// requeue: the pod's cycle failed (AddUnschedulableIfNotPresent re-stamps it).
func (t *tracker) requeue(uid types.UID) {
	t.mu.Lock()
	t.queued[uid] = t.tick
	t.tick++
	t.failed[uid] = struct{}{}
	t.mu.Unlock()
}

// popped: the pod's cycle starts, so it left whichever sub-queue held it.
func (t *tracker) popped(uid types.UID) {
	t.mu.Lock()
	delete(t.failed, uid)
	t.mu.Unlock()
}

// queueKeys returns each pod's stamp (-1: not seen yet) and whether it waits after a failed cycle.
func (t *tracker) queueKeys(pods []*v1.Pod) ([]int64, []bool) {
	t.mu.Lock()
	defer t.mu.Unlock()
	at := make([]int64, len(pods))
	bad := make([]bool, len(pods))
	for i, p := range pods {
		at[i] = -1
		if v, ok := t.queued[p.UID]; ok {
			at[i] = v
		}
		_, bad[i] = t.failed[p.UID]
	}
	return at, bad
}

func (t *tracker) mark(node string) {
	if node == "" {
		return
	}
	t.mu.Lock()
	t.marks[node] = markTTL
	t.mu.Unlock()
}

// take returns the marked nodes and ages the marks; keep(name) re-arms a mark whose NodeInfo has not
// moved yet (its event may not have reached the cache).
func (t *tracker) take() []string {
	t.mu.Lock()
	defer t.mu.Unlock()
	out := make([]string, 0, len(t.marks))
	for n, left := range t.marks {
		out = append(out, n)
		if left <= 1 {
			delete(t.marks, n)
			t.full = true
		} else {
			t.marks[n] = left - 1
		}
	}
	return out
}

// takeFull reports (and clears) a pending full scan.
func (t *tracker) takeFull() bool {
	t.mu.Lock()
	defer t.mu.Unlock()
	f := t.full
	t.full = false
	return f
}

// nominate records a node that may hold nominated pods.
func (t *tracker) nominate(node string) {
	if node == "" {
		return
	}
	t.mu.Lock()
	t.noms[node] = struct{}{}
	t.mu.Unlock()
}

// nominations returns the recorded nodes and clears the record.
func (t *tracker) nominations() []string {
	t.mu.Lock()
	defer t.mu.Unlock()
	out := make([]string, 0, len(t.noms))
	for n := range t.noms {
		out = append(out, n)
		delete(t.noms, n)
	}
	return out
}

// peek returns the marked nodes without aging the marks.
func (t *tracker) peek() []string {
	t.mu.Lock()
	defer t.mu.Unlock()
	out := make([]string, 0, len(t.marks))
	for n := range t.marks {
		out = append(out, n)
	}
	return out
}

// settle drops the mark of a node whose change was applied.
func (t *tracker) settle(node string) {
	t.mu.Lock()
	delete(t.marks, node)
	t.mu.Unlock()
}

func podOf(obj interface{}) *v1.Pod {
	switch o := obj.(type) {
	case *v1.Pod:
		return o
	case cache.DeletedFinalStateUnknown:
		if p, ok := o.Obj.(*v1.Pod); ok {
			return p
		}
	}
	return nil
}

func nodeOf(obj interface{}) *v1.Node {
	switch o := obj.(type) {
	case *v1.Node:
		return o
	case cache.DeletedFinalStateUnknown:
		if n, ok := o.Obj.(*v1.Node); ok {
			return n
		}
	}
	return nil
}

// watch registers the informer handlers (FrameworkHandle.SharedInformerFactory, interface.go:515).
// Without informers every sync compares every generation.
func (g *GpuEval) watch() {
	f := g.h.SharedInformerFactory()
	if f == nil {
		g.exact = true
		return
	}
	t := g.track
	onPod := func(objs ...interface{}) {
		for _, o := range objs {
			if p := podOf(o); p != nil {
				t.mark(p.Spec.NodeName)
				if p.Spec.NodeName == "" {
					t.nominate(p.Status.NominatedNodeName)
				}
			}
		}
	}
	// the queue clock follows the last object of each event
	onQueue := func(o interface{}, deleted bool) {
		if p := podOf(o); p != nil {
			if deleted || p.Spec.NodeName != "" {
				t.dequeue(p.UID)
			} else {
				t.enqueue(p.UID)
			}
		}
	}
	f.Core().V1().Pods().Informer().AddEventHandler(cache.ResourceEventHandlerFuncs{
		AddFunc:    func(o interface{}) { onPod(o); onQueue(o, false) },
		UpdateFunc: func(o, n interface{}) { onPod(o, n); onQueue(n, false) },
		DeleteFunc: func(o interface{}) { onPod(o); onQueue(o, true) },
	})
	onNode := func(objs ...interface{}) {
		for _, o := range objs {
			if n := nodeOf(o); n != nil {
				t.mark(n.Name)
			}
		}
	}
	f.Core().V1().Nodes().Informer().AddEventHandler(cache.ResourceEventHandlerFuncs{
		AddFunc:    func(o interface{}) { onNode(o) },
		UpdateFunc: func(o, n interface{}) { onNode(o, n) },
		DeleteFunc: func(o interface{}) { onNode(o) },
	})
}
