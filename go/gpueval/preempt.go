package gpueval

// Nominated pods and preemption on the device (SURVEY.md 8(f)3).
//
// PreFilter copies the PreemptHandle's PodNominator into the engine (kgpu_set_nominated), so the
// cycle's status words already hold podPassesFiltersOnNode's two-pass verdict
// (generic_scheduler.go:526-615).  Preemption: this reference version runs genericScheduler.Preempt
// in-tree before the PostFilter plugins (scheduler.go:543-562), and Preempt re-runs the Filter
// plugins on NodeInfo clones with victims removed, which a status-word lookup cannot answer.  The
// drop-in is SelectVictims: the body of Preempt after its eligibility checks
// (generic_scheduler.go:263-301), called from a two-line patch of genericScheduler.Preempt or from
// PostFilter once preemption moves there (the TODO at scheduler.go:548).

/*
#include "kgpu.h"
*/
import "C"

import (
	"context"
	"fmt"

	v1 "k8s.io/api/core/v1"
	policy "k8s.io/api/policy/v1beta1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/labels"
	podutil "k8s.io/kubernetes/pkg/api/v1/pod"
	framework "k8s.io/kubernetes/pkg/scheduler/framework/v1alpha1"
	"k8s.io/kubernetes/pkg/scheduler/util"
)

// syncNominated sends NominatedPodsForNode of every listed node to the engine.
func (g *GpuEval) syncNominated(a *arena) error {
	ph := g.h.PreemptHandle()
	if ph == nil {
		return nil
	}
	var noms []C.kgpu_nominated
	var recs []C.kgpu_pod_query
	p := &pools{}
	for i, name := range g.mir.names {
		for _, np := range ph.NominatedPodsForNode(name) {
			q, err := g.comp.compilePod(np, p)
			if err != nil {
				return err
			}
			noms = append(noms, C.kgpu_nominated{node: C.int32_t(i), item: C.int32_t(len(recs))})
			recs = append(recs, q)
		}
	}
	if len(noms) == 0 && !g.nominated {
		return nil
	}
	g.nominated = len(noms) > 0
	return g.eng.setNominated(noms, recs, p.toC(a))
}

// pdbsOf: indices of the PodDisruptionBudgets selecting the pod, in the caller's order
// (filterPodsWithPDBViolation, generic_scheduler.go:886-905: same namespace, a non-empty selector
// matching the pod's labels; a label-less pod matches none).
func pdbsOf(pod *v1.Pod, pdbs []*policy.PodDisruptionBudget) []int {
	var out []int
	if len(pod.Labels) == 0 {
		return nil
	}
	for j, pdb := range pdbs {
		if pdb.Namespace != pod.Namespace {
			continue
		}
		sel, err := metav1.LabelSelectorAsSelector(pdb.Spec.Selector)
		if err != nil || sel.Empty() || !sel.Matches(labels.Set(pod.Labels)) {
			continue
		}
		out = append(out, j)
	}
	return out
}

// SelectVictims runs selectNodesForPreemption + pickOneNodeForPreemption for a pod whose cycle
// ended in a FitError (its PreFilter ran on this snapshot).  Returns the node and the victims, in
// Victims.Pods order; "" when no node can make room.
func (g *GpuEval) SelectVictims(ctx context.Context, pod *v1.Pod, pdbs []*policy.PodDisruptionBudget) (string, []*v1.Pod, error) {
	list, err := g.h.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return "", nil, err
	}
	var a arena
	defer a.free()
	p := &pools{}
	q, err := g.comp.compilePod(pod, p)
	if err != nil {
		return "", nil, err
	}
	if sel := g.defaultSelector(pod); sel != nil {
		if q.dpts, err = g.comp.labelSelector(p, sel); err != nil {
			return "", nil, err
		}
	}
	prio := podutil.GetPodPriority(pod)
	var victims []C.kgpu_victim
	var recs []C.kgpu_pod_query
	var pods []*v1.Pod
	var victimPDBs [][]int
	// Preempt lists every PDB of the cluster (labels.Everything()), but filterPodsWithPDBViolation
	// only touches the ones that select a potential victim, walking them in order: the engine gets
	// that subset, renumbered in the same order, so its 64-bit masks cover any cluster.
	used := map[int]int{}
	var usedOrder []int
	for _, ni := range list {
		idx, ok := g.mir.index[ni.Node().Name]
		if !ok {
			continue
		}
		for _, pi := range ni.Pods { // NodeInfo.Pods order: MoreImportantPod ties keep it
			if podutil.GetPodPriority(pi.Pod) >= prio {
				continue
			}
			slot, ok := g.mir.slots[pi.Pod.UID]
			if !ok {
				// a pod the device mirror does not hold: its effects would be read from another
				// pod's slot; resync before preempting
				g.mir = nil
				return "", nil, fmt.Errorf("gpueval: pod %s/%s is not in the device mirror (resynced; retry)",
					pi.Pod.Namespace, pi.Pod.Name)
			}
			r, err := g.comp.compilePod(pi.Pod, p)
			if err != nil {
				return "", nil, err
			}
			js := pdbsOf(pi.Pod, pdbs)
			for _, j := range js {
				if _, seen := used[j]; !seen {
					used[j] = -1
					usedOrder = append(usedOrder, j)
				}
			}
			victims = append(victims, C.kgpu_victim{node: C.int32_t(idx), slot: C.int32_t(slot),
				item: C.int32_t(len(recs)), start_time: C.int64_t(util.GetPodStartTime(pi.Pod).UnixNano())})
			victimPDBs = append(victimPDBs, js)
			recs = append(recs, r)
			pods = append(pods, pi.Pod)
		}
	}
	sortInts(usedOrder)
	if len(usedOrder) > 64 {
		return "", nil, fmt.Errorf("gpueval: %d PodDisruptionBudgets select potential victims (the engine takes 64)", len(usedOrder))
	}
	allowed := make([]int32, 0, len(usedOrder))
	for k, j := range usedOrder {
		used[j] = k
		allowed = append(allowed, pdbs[j].Status.DisruptionsAllowed)
	}
	for i, js := range victimPDBs {
		var m uint64
		for _, j := range js {
			m |= 1 << uint(used[j])
		}
		victims[i].pdb_mask = C.uint64_t(m)
	}
	cq := cQueries(&a, []C.kgpu_pod_query{q})
	out, vout, chosen, err := g.eng.selectVictims(cq, p.toC(&a), victims, recs, allowed, len(g.mir.names))
	if err != nil || chosen < 0 {
		return "", nil, err
	}
	o := out[chosen]
	res := make([]*v1.Pod, 0, int(o.n_victims))
	for k := 0; k < int(o.n_victims); k++ {
		res = append(res, pods[vout[int(o.first)+k]])
	}
	return g.mir.names[chosen], res, nil
}

func sortInts(x []int) {
	for i := 1; i < len(x); i++ {
		for k := i; k > 0 && x[k] < x[k-1]; k-- {
			x[k], x[k-1] = x[k-1], x[k]
		}
	}
}

// PostFilter (interface.go:276-290): the device's preemption choice as the nominated node.  In
// this reference version it runs after the in-tree Preempt (scheduler.go:543-562); victims are
// deleted by the caller that owns the client (sched.podPreemptor), as Preempt's caller does.
func (g *GpuEval) PostFilter(ctx context.Context, cs *framework.CycleState, pod *v1.Pod,
	m framework.NodeToStatusMap) (*framework.PostFilterResult, *framework.Status) {
	node, _, err := g.SelectVictims(ctx, pod, nil)
	if err != nil {
		return nil, framework.NewStatus(framework.Error, err.Error())
	}
	if node == "" {
		return nil, framework.NewStatus(framework.Unschedulable)
	}
	return &framework.PostFilterResult{NominatedNodeName: node}, nil
}
