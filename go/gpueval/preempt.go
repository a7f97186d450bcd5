package gpueval

// Nominated pods and preemption on the device (SURVEY.md 8(f)3).
//
// PreFilter copies the PreemptHandle's PodNominator into the engine (kgpu_set_nominated), so the
// cycle's status words already hold podPassesFiltersOnNode's two-pass verdict
// (generic_scheduler.go:526-615).
//
// Preemption.  This reference version runs genericScheduler.Preempt in-tree, before the PostFilter
// plugins (scheduler.go:543-562), and only that path evicts: sched.preempt deletes the victims and
// records the nomination.  A PostFilter plugin here can only return a NominatedNodeName, which would
// nominate the pod to a node whose victims nobody deletes -- so this package ships no PostFilter.
// Preempt's candidate search, selectNodesForPreemption (generic_scheduler.go:845-876), re-runs the
// Filter plugins on NodeInfo clones with victims removed, which a status-word lookup cannot answer.
// The drop-in replaces exactly that call (INTEGRATION.md section 9):
//
//	if gp := gpueval.ForFramework(prof.Framework); gp != nil {
//		nodeNameToVictims, err = gp.SelectNodesForPreemption(ctx, pod, potentialNodes, pdbs)
//	} else {
//		nodeNameToVictims, err = selectNodesForPreemption(ctx, prof, g.podNominator, state, pod, potentialNodes, pdbs)
//	}
//
// so Preempt keeps its own eligibility checks, the real PDB list (g.pdbLister), the extenders
// (processPreemptionWithExtenders) and pickOneNodeForPreemption.  ForFramework finds the plugin by
// the FrameworkHandle New received, which is the *framework profile.Profile embeds.

/*
#include "kgpu.h"
*/
import "C"

import (
	"context"
	"fmt"
	"sync"

	v1 "k8s.io/api/core/v1"
	policy "k8s.io/api/policy/v1beta1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/labels"
	extenderv1 "k8s.io/kube-scheduler/extender/v1"
	podutil "k8s.io/kubernetes/pkg/api/v1/pod"
	framework "k8s.io/kubernetes/pkg/scheduler/framework/v1alpha1"
	"k8s.io/kubernetes/pkg/scheduler/util"
)

// The plugins New built, by the FrameworkHandle they were built with (one per profile).
var (
	registryMu sync.Mutex
	registry   = map[framework.FrameworkHandle]*GpuEval{}
)

func register(h framework.FrameworkHandle, g *GpuEval) {
	registryMu.Lock()
	registry[h] = g
	registryMu.Unlock()
}

func unregister(g *GpuEval) {
	registryMu.Lock()
	for h, x := range registry {
		if x == g {
			delete(registry, h)
		}
	}
	registryMu.Unlock()
}

// ForFramework returns the GpuEval of the profile whose framework is fw (profile.Profile.Framework),
// or nil when that profile does not run one.
func ForFramework(fw framework.FrameworkHandle) *GpuEval {
	if fw == nil {
		return nil
	}
	registryMu.Lock()
	defer registryMu.Unlock()
	return registry[fw]
}

// syncNominated sends the PodNominator's pods to the engine.  It asks NominatedPodsForNode only
// about the nodes that may hold nominated pods (track.go: the informers' NominatedNodeName, the
// candidates of this plugin's preemptions) and the nodes that held some at the last sync, so a cycle
// costs O(nominated) map operations, not one per listed node.
func (g *GpuEval) syncNominated(a *arena) error {
	ph := g.h.PreemptHandle()
	if ph == nil {
		return nil
	}
	cand := map[string]struct{}{}
	for _, n := range g.nomLast {
		cand[n] = struct{}{}
	}
	for _, n := range g.track.nominations() {
		cand[n] = struct{}{}
	}
	if len(cand) == 0 && !g.nominated {
		return nil
	}
	idx := make([]int32, 0, len(cand))
	for n := range cand {
		if i, ok := g.mir.index[n]; ok {
			idx = append(idx, i)
		}
	}
	sortInt32s(idx) // Snapshot.List() order, as a walk over the list would send them
	var noms []C.kgpu_nominated
	var recs []C.kgpu_pod_query
	ps, err := newPoolSet()
	if err != nil {
		return err
	}
	a.onFree(ps.free)
	g.nomLast = g.nomLast[:0]
	for _, i := range idx {
		name := g.mir.names[i]
		pods := ph.NominatedPodsForNode(name)
		if len(pods) > 0 {
			g.nomLast = append(g.nomLast, name)
		}
		for _, np := range pods {
			q, err := g.comp.compilePod(np, nil, ps) // addNominatedPods reads no DefaultSelector
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
	return g.eng.setNominated(noms, recs, ps.toC(a))
}

func sortInt32s(x []int32) {
	for i := 1; i < len(x); i++ {
		for k := i; k > 0 && x[k] < x[k-1]; k-- {
			x[k], x[k-1] = x[k-1], x[k]
		}
	}
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

// SelectNodesForPreemption replaces selectNodesForPreemption (generic_scheduler.go:845-876) for a pod
// whose cycle ended in a FitError: every node of potentialNodes where the pod fits once lower-priority
// pods are removed, with the victims selectVictimsOnNode keeps (Victims.Pods order) and the PDB
// violations among them.  pdbs: the cluster's PodDisruptionBudgets, as Preempt lists them.
func (g *GpuEval) SelectNodesForPreemption(ctx context.Context, pod *v1.Pod, potentialNodes []*framework.NodeInfo,
	pdbs []*policy.PodDisruptionBudget) (map[string]*extenderv1.Victims, error) {
	out, _, err := g.selectOnDevice(pod, potentialNodes, pdbs)
	return out, err
}

// SelectVictims is SelectNodesForPreemption over every listed node followed by the device's
// pickOneNodeForPreemption (ties in Snapshot.List() order): the node and its victims, "" when no
// node can make room.  For callers that keep no extenders (tools, tests).
func (g *GpuEval) SelectVictims(ctx context.Context, pod *v1.Pod, pdbs []*policy.PodDisruptionBudget) (string, []*v1.Pod, error) {
	list, err := g.h.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return "", nil, err
	}
	out, chosen, err := g.selectOnDevice(pod, list, pdbs)
	if err != nil || chosen == "" {
		return "", nil, err
	}
	return chosen, out[chosen].Pods, nil
}

// selectOnDevice: one kgpu_select_victims call over the lower-priority pods of `nodes`.  Nodes outside
// `nodes` get no potential victims, so they keep failing the filters they failed this cycle and are
// never candidates.  Returns the candidates and the device's pick.
func (g *GpuEval) selectOnDevice(pod *v1.Pod, nodes []*framework.NodeInfo,
	pdbs []*policy.PodDisruptionBudget) (map[string]*extenderv1.Victims, string, error) {
	list := nodes
	var a arena
	defer a.free()
	ps, err := newPoolSet()
	if err != nil {
		return nil, "", err
	}
	a.onFree(ps.free)
	q, err := g.comp.compilePod(pod, g.defaultSelector(pod), ps)
	if err != nil {
		return nil, "", err
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
				return nil, "", fmt.Errorf("gpueval: pod %s/%s is not in the device mirror (resynced; retry)",
					pi.Pod.Namespace, pi.Pod.Name)
			}
			r, err := g.comp.compilePod(pi.Pod, nil, ps)
			if err != nil {
				return nil, "", err
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
		return nil, "", fmt.Errorf("gpueval: %d PodDisruptionBudgets select potential victims (the engine takes 64)", len(usedOrder))
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
	out, vout, chosen, err := g.eng.selectVictims(cq, ps.toC(&a), victims, recs, allowed, len(g.mir.names))
	if err != nil {
		return nil, "", err
	}
	res := map[string]*extenderv1.Victims{}
	for _, ni := range list {
		idx, ok := g.mir.index[ni.Node().Name]
		if !ok || out[idx].fits == 0 {
			continue
		}
		o := out[idx]
		vs := make([]*v1.Pod, 0, int(o.n_victims))
		for k := 0; k < int(o.n_victims); k++ {
			vs = append(vs, pods[vout[int(o.first)+k]])
		}
		res[ni.Node().Name] = &extenderv1.Victims{Pods: vs, NumPDBViolations: int64(o.num_pdb_violations)}
		// the scheduler nominates the pod to one of these before the status update reaches the
		// informer: the next cycles ask the PodNominator about all of them (syncNominated)
		g.track.nominate(ni.Node().Name)
	}
	name := ""
	if chosen >= 0 {
		name = g.mir.names[chosen]
	}
	return res, name, nil
}

func sortInts(x []int) {
	for i := 1; i < len(x); i++ {
		for k := i; k > 0 && x[k] < x[k-1]; k-- {
			x[k], x[k-1] = x[k-1], x[k]
		}
	}
}
