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

// pdbMask: the PodDisruptionBudgets selecting the pod (filterPodsWithPDBViolation,
// generic_scheduler.go:886-905).
func pdbMask(pod *v1.Pod, pdbs []*policy.PodDisruptionBudget) uint64 {
	var m uint64
	if len(pod.Labels) == 0 {
		return 0
	}
	for j, pdb := range pdbs {
		if j >= 64 || pdb.Namespace != pod.Namespace {
			continue
		}
		sel, err := metav1.LabelSelectorAsSelector(pdb.Spec.Selector)
		if err != nil || sel.Empty() || !sel.Matches(labels.Set(pod.Labels)) {
			continue
		}
		m |= 1 << uint(j)
	}
	return m
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
	for _, ni := range list {
		idx, ok := g.mir.index[ni.Node().Name]
		if !ok {
			continue
		}
		for _, pi := range ni.Pods { // NodeInfo.Pods order: MoreImportantPod ties keep it
			if podutil.GetPodPriority(pi.Pod) >= prio {
				continue
			}
			r, err := g.comp.compilePod(pi.Pod, p)
			if err != nil {
				return "", nil, err
			}
			victims = append(victims, C.kgpu_victim{node: C.int32_t(idx), slot: C.int32_t(g.mir.slots[pi.Pod.UID]),
				item: C.int32_t(len(recs)), start_time: C.int64_t(util.GetPodStartTime(pi.Pod).UnixNano()),
				pdb_mask: C.uint64_t(pdbMask(pi.Pod, pdbs))})
			recs = append(recs, r)
			pods = append(pods, pi.Pod)
		}
	}
	allowed := make([]int32, 0, len(pdbs))
	for _, pdb := range pdbs {
		allowed = append(allowed, pdb.Status.DisruptionsAllowed)
	}
	cq := cslice(&a, []C.kgpu_pod_query{q})
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
