package gpueval

// GpuEval: one out-of-tree plugin that replaces the filter / score plugins of a profile with the
// device (SURVEY.md 8(b) adapter pattern).  PreFilter syncs the device mirror with the Snapshot
// the cycle runs on, compiles the pod and runs the whole cycle in one C call; Filter and Score are
// lock-free lookups in the cycle record, safe under parallelize.Until's 16 goroutines.
//
// Two score modes (profileArgs.Mode):
//   select: one score plugin (weight 1) returns 100 for the device-chosen node and 0 otherwise,
//           so the reference selectHost (generic_scheduler.go:217-238) picks the device's node;
//   shadow: one GPU score plugin per replaced score plugin (ShadowPlugins, shadow.go), each returning
//           that plugin's device-normalized 0-100 value; the profile gives them the reference weights,
//           so the framework's range check, weighting and sum (framework.go:632-648) and the reference
//           selectHost run unchanged on the device's per-plugin scores.
//
// Reserve / Unreserve need no device call: cache.AssumePod / ForgetPod update the NodeInfo, and the
// next PreFilter's generation diff (soa.go) sends NodeInfo.AddPod / RemovePod by UID; they mark the
// node for that diff (track.go).

/*
#include "kgpu.h"
#include "kgpu_compile.h"
*/
import "C"

import (
	"context"
	"fmt"
	"sort"
	"sync/atomic"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/labels"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/apimachinery/pkg/types"
	v1helper "k8s.io/kubernetes/pkg/apis/core/v1/helper"
	framework "k8s.io/kubernetes/pkg/scheduler/framework/v1alpha1"
)

const Name = "GpuEval"

const stateKey framework.StateKey = Name

// profileArgs: the replaced plugins and their args (apis/config/types.go:115-239,
// types_pluginargs.go), forwarded into kgpu_config.
type profileArgs struct {
	Filters                []string
	Scores                 []struct{ Name string; Weight int64 }
	LeastResources         map[string]int64
	MostResources          map[string]int64
	RTCRResources          map[string]int64
	RTCRShape              [][2]int64 // (utilization, score 0-10)
	HardPodAffinityWeight  int32
	PercentageOfNodesToScore int32
	TieBreakSeed           uint64
	Mode                   string // "select" or "shadow"
	ExactSync              bool   // compare every NodeInfo generation at every sync (track.go)
	BatchAhead             int    // > 1: schedule the pod with the next BatchAhead-1 queued pods (ahead.go)
	// DefaultConstraints: PodTopologySpreadArgs.DefaultConstraints (apis/config/types_pluginargs.go),
	// applied with the pod's DefaultSelector to a pod without constraints (podtopologyspread/common.go:44-72).
	DefaultConstraints     []v1.TopologySpreadConstraint
	// RunAllFilters mirrors the framework's runAllFilters (framework.go:90,155-160,494), which the
	// scheduler sets from the legacy Policy's AlwaysCheckAllPredicates (factory.go:107,278-281): every
	// filter plugin runs on every node and Filter returns the merged status with every failing
	// plugin's reasons (KGPU_OPT_RUN_ALL_FILTERS).  Set it together with that Policy field.
	RunAllFilters          bool
	ignoredResources       map[string]struct{}
}

var filterIDs = map[string]int32{"NodeUnschedulable": C.KGPU_F_NODE_UNSCHEDULABLE, "NodeResourcesFit": C.KGPU_F_NODE_RESOURCES_FIT,
	"NodeName": C.KGPU_F_NODE_NAME, "NodePorts": C.KGPU_F_NODE_PORTS, "NodeAffinity": C.KGPU_F_NODE_AFFINITY,
	"TaintToleration": C.KGPU_F_TAINT_TOLERATION, "PodTopologySpread": C.KGPU_F_POD_TOPOLOGY_SPREAD,
	"InterPodAffinity": C.KGPU_F_INTER_POD_AFFINITY}

var scoreIDs = map[string]int32{"NodeResourcesBalancedAllocation": C.KGPU_S_BALANCED_ALLOCATION,
	"ImageLocality": C.KGPU_S_IMAGE_LOCALITY, "InterPodAffinity": C.KGPU_S_INTER_POD_AFFINITY,
	"NodeResourcesLeastAllocated": C.KGPU_S_LEAST_ALLOCATED, "NodeAffinity": C.KGPU_S_NODE_AFFINITY,
	"NodePreferAvoidPods": C.KGPU_S_NODE_PREFER_AVOID_PODS, "PodTopologySpread": C.KGPU_S_POD_TOPOLOGY_SPREAD,
	"DefaultPodTopologySpread": C.KGPU_S_DEFAULT_POD_TOPOLOGY_SPREAD, "TaintToleration": C.KGPU_S_TAINT_TOLERATION,
	"NodeResourcesMostAllocated": C.KGPU_S_MOST_ALLOCATED, "RequestedToCapacityRatio": C.KGPU_S_REQUESTED_TO_CAPACITY_RATIO,
	"NodeResourceLimits": C.KGPU_S_RESOURCE_LIMITS}

func sortedNames(m map[string]int64) []string {
	out := make([]string, 0, len(m))
	for r := range m {
		out = append(out, r)
	}
	sort.Strings(out)
	return out
}

func sortStrings(x []string) { sort.Strings(x) }

// config builds kgpu_config (kubernetes-1_amd/kgpu/compile.py Compiler.config).
func (c *compiler) config() *C.kgpu_config {
	p := c.prof
	var cfg C.kgpu_config
	cfg.abi_version = C.KGPU_ABI_VERSION
	for _, f := range p.Filters {
		if id, ok := filterIDs[f]; ok {
			cfg.filters[cfg.n_filters] = C.int32_t(id)
			cfg.n_filters++
		}
	}
	for _, s := range p.Scores {
		cfg.scores[cfg.n_scores] = C.int32_t(scoreIDs[s.Name])
		w := s.Weight
		if w == 0 {
			w = 1
		}
		cfg.score_weights[cfg.n_scores] = C.int64_t(w)
		cfg.n_scores++
	}
	res := func(name string) int32 {
		switch name {
		case "cpu":
			return 0
		case "memory":
			return 1
		case "ephemeral-storage":
			return 2
		}
		if col := c.scalarColumn(name); col >= 0 && v1helper.IsScalarResourceName(v1.ResourceName(name)) {
			return 3 + col // the compiler gave every profile resource a column up front
		}
		return -1
	}
	fill := func(m map[string]int64, arr *[8]C.kgpu_resource_weight, n *C.int32_t) {
		names := make([]string, 0, len(m))
		for r := range m {
			names = append(names, r)
		}
		sort.Strings(names)
		for i, r := range names {
			arr[i] = C.kgpu_resource_weight{resource: C.int32_t(res(r)), weight: C.int32_t(m[r])}
		}
		*n = C.int32_t(len(names))
	}
	fill(p.LeastResources, &cfg.least, &cfg.n_least)
	fill(p.MostResources, &cfg.most, &cfg.n_most)
	fill(p.RTCRResources, &cfg.rtcr, &cfg.n_rtcr)
	for i, pt := range p.RTCRShape {
		cfg.shape[i] = C.kgpu_shape_point{utilization: C.int64_t(pt[0]), score: C.int64_t(pt[1] * 10)}
	}
	cfg.n_shape = C.int32_t(len(p.RTCRShape))
	cfg.hard_pod_affinity_weight = C.int32_t(p.HardPodAffinityWeight)
	cfg.percentage_of_nodes_to_score = C.int32_t(p.PercentageOfNodesToScore)
	cfg.seed = C.uint64_t(p.TieBreakSeed)
	return &cfg
}

// cycle is the per-pod state read by Filter and Score (and by the shadow score plugins).
type cycle struct {
	words  []uint32           // per-node filter status words (node index order)
	all    []uint32           // RunAllFilters: [filter position][node] each plugin's own word
	norm   map[int32][]int64  // shadow mode: per score plugin id, the device-normalized 0-100 value per node
	index  map[string]int32   // node name -> node index of this cycle's mirror
	chosen int32              // device-selected node index, -1 = FitError
	rq     *reasonQuery       // the pod's C query for kgpu_filter_reasons (owned by GpuEval.rq)
}

func (c *cycle) Clone() framework.StateData { return c }

type GpuEval struct {
	h         framework.FrameworkHandle
	prof      *profileArgs
	eng       *engine
	comp      *compiler
	mir       *mirror
	seq       int64
	nominated bool     // the engine holds a non-empty nominator
	nomLast   []string // nodes that held nominated pods at the last sync (preempt.go syncNominated)
	ahead     *ahead   // batch-ahead (ahead.go; profileArgs.BatchAhead > 1, select mode)
	track     *tracker // nodes whose NodeInfo may have moved since the last sync (track.go)
	exact     bool     // compare every generation at every sync
	syncs     int
	// the pod of the last PreFilter, and whether it reached Reserve (track.go queue clock)
	lastPod types.UID
	lastRes bool
	rq      *reasonQuery // the last diagnostic cycle's query, freed by the next PreFilter
}

func (g *GpuEval) Name() string { return Name }

func readCycle(cs *framework.CycleState) (*cycle, error) {
	d, err := cs.Read(stateKey)
	if err != nil {
		return nil, err
	}
	c, ok := d.(*cycle)
	if !ok {
		return nil, fmt.Errorf("%+v convert to gpueval.cycle error", d)
	}
	return c, nil
}

// syncSnapshot brings the device mirror to the Snapshot of this cycle: a delta when the
// dictionaries can absorb the changes, a full upload otherwise.
func (g *GpuEval) syncSnapshot() error {
	list, err := g.h.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return err
	}
	var a arena
	defer a.free()
	if g.mir != nil {
		b, err := g.deltaFromSnapshot(list, &a)
		if err == nil {
			g.mir.gen++
			var slots []int32
			slots, err = g.eng.applyDelta(b, g.mir.gen)
			if err == nil {
				g.mir.recordSlots(slots)
				return nil
			}
		}
		if err != errNeedsUpload {
			// the engine marks a failed batch's mirror invalid: rebuild it from scratch
			g.mir = nil
		}
	}
	return g.upload(list, &a)
}

// upload compiles the whole Snapshot.List() into kgpu_snapshot columns (a fresh compiler: the
// dictionaries of a new upload epoch).
func (g *GpuEval) upload(list []*framework.NodeInfo, a *arena) error {
	c, err := newCompiler(g.prof)
	if err != nil {
		return err
	}
	for _, ni := range list {
		if err := c.registerNode(ni.Node()); err != nil {
			c.close()
			return err
		}
		for _, pi := range ni.Pods {
			if err := c.registerPod(pi.Pod); err != nil {
				c.close()
				return err
			}
		}
	}
	c.dictAdd(C.KGPU_DICT_NAMESPACE, 0, "")
	g.track.take() // a full upload covers every mark
	if g.eng == nil {
		eng, err := newEngine(c.config())
		if err != nil {
			c.close()
			return err
		}
		if g.prof.RunAllFilters {
			if err := eng.setOption(C.KGPU_OPT_RUN_ALL_FILTERS, 1); err != nil {
				eng.close()
				c.close()
				return err
			}
		}
		g.eng = eng
	}
	g.comp.close()
	g.comp = c
	m := &mirror{index: map[string]int32{}, gens: map[string]int64{}, nodes: map[string]*v1.Node{},
		pods: map[string]map[types.UID]*v1.Pod{}, uids: map[types.UID]int64{}, slots: map[types.UID]int32{},
		res: map[string]nodeRes{}}
	m.genAt = make([]int64, len(list))
	for i, ni := range list {
		m.genAt[i] = ni.Generation
	}
	if len(list) > 0 {
		m.listData = unsafe.Pointer(&list[0])
	}
	if g.mir != nil {
		m.uids, m.nextUID, m.gen = g.mir.uids, g.mir.nextUID, g.mir.gen
	}
	s, err := g.snapshotSoA(list, m, a)
	if err != nil {
		return err
	}
	m.gen++
	g.mir = m
	if err := g.eng.uploadSnapshot(s, m.gen); err != nil {
		return err
	}
	return g.prepareQueue()
}

// prepareQueue registers the pod classes of the unassigned pods the informer holds (at most
// prepareMax): a new upload epoch starts with empty class tables, and the first cycle of each class
// would otherwise pay its count (kgpu_prepare_pods).
const prepareMax = 512

func (g *GpuEval) prepareQueue() error {
	f := g.h.SharedInformerFactory()
	if f == nil {
		return nil
	}
	all, err := f.Core().V1().Pods().Lister().List(labels.Everything())
	if err != nil {
		return nil
	}
	ps, err := newPoolSet()
	if err != nil {
		return err
	}
	defer ps.free()
	var qs []C.kgpu_pod_query
	for _, p := range all {
		if p.Spec.NodeName != "" || p.DeletionTimestamp != nil {
			continue
		}
		q, err := g.comp.compilePod(p, g.defaultSelector(p), ps)
		if err != nil {
			continue // that pod's own cycle reports it
		}
		qs = append(qs, q)
		if len(qs) == prepareMax {
			break
		}
	}
	var a arena
	defer a.free()
	return g.eng.preparePods(qs, ps.toC(&a))
}

// snapshotSoA compiles the list's nodes and their NodeInfos' pods (kgpu_compile_snapshot: the node
// columns, NodeInfo.AddPod of every pod, the pods' label rows and affinity terms).  The list is
// uploaded once per distinct node; a list holding a NodeInfo twice is aliased by the next delta's
// order (kgpu_delta_batch.order).  Pod-table slots follow the pods' order here.
func (g *GpuEval) snapshotSoA(list []*framework.NodeInfo, m *mirror, a *arena) (*C.kgpu_snapshot, error) {
	c := g.comp
	seen := map[string]bool{}
	var nodes []*v1.Node
	var existing []*v1.Pod
	var hosts []string
	var uids []int64
	for _, ni := range list {
		n := ni.Node()
		if seen[n.Name] {
			continue
		}
		seen[n.Name] = true
		m.names = append(m.names, n.Name)
		m.index[n.Name] = int32(len(nodes))
		m.gens[n.Name] = ni.Generation
		m.nodes[n.Name] = n
		m.res[n.Name] = resOf(ni)
		m.pods[n.Name] = map[types.UID]*v1.Pod{}
		nodes = append(nodes, n)
		for _, pi := range ni.Pods {
			m.pods[n.Name][pi.Pod.UID] = pi.Pod
			m.slots[pi.Pod.UID] = int32(len(existing))
			existing = append(existing, pi.Pod)
			hosts = append(hosts, n.Name)
			uids = append(uids, m.uid(pi.Pod.UID))
		}
	}
	s, err := c.snapshot(nodes, existing, hosts, uids, a)
	if err != nil {
		return nil, err
	}
	for _, n := range nodes {
		for _, kv := range c.nodeLabelIDs(n) {
			m.labels.add(kv[0], kv[1], 1)
		}
	}
	return s, nil
}

// PreFilter: sync the device mirror to this cycle's Snapshot, compile the pod, run the cycle.  With
// batch-ahead the cycle may be served from (or start) a batch of the pods the queue pops next.
func (g *GpuEval) PreFilter(ctx context.Context, cs *framework.CycleState, pod *v1.Pod) *framework.Status {
	seq := atomic.AddInt64(&g.seq, 1) - 1
	if g.lastPod != "" && !g.lastRes {
		g.track.requeue(g.lastPod) // that cycle failed before Reserve (scheduler.go:535-576 recordSchedulingFailure)
	}
	g.lastPod, g.lastRes = pod.UID, false
	g.track.popped(pod.UID)
	if g.ahead != nil {
		res, ok, err := g.serveAhead(pod, seq)
		if err != nil {
			return framework.NewStatus(framework.Error, err.Error())
		}
		if ok && res.node >= 0 {
			cs.Write(stateKey, &cycle{chosen: int32(res.node), index: g.mir.index})
			return nil
		}
		if ok {
			// unschedulable in the batch: its FitError statuses come from a diagnostic cycle on the
			// state without the speculation
			if err := g.invalidate(); err != nil {
				return framework.NewStatus(framework.Error, err.Error())
			}
		}
	}
	if err := g.syncSnapshot(); err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	var a arena
	defer a.free()
	if err := g.syncNominated(&a); err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	ps, err := newPoolSet()
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	kept := false // ps passes to the cycle's reasonQuery
	defer func() {
		if !kept {
			ps.free()
		}
	}()
	q, err := g.comp.compilePod(pod, g.defaultSelector(pod), ps)
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	if g.ahead != nil && !g.nominated {
		if res, ok, err := g.startBatch(pod, q, ps, seq); err != nil {
			return framework.NewStatus(framework.Error, err.Error())
		} else if ok && res.node >= 0 {
			cs.Write(stateKey, &cycle{chosen: int32(res.node), index: g.mir.index})
			return nil
		} else if ok {
			if err := g.invalidate(); err != nil { // FitError: statuses from a diagnostic cycle
				return framework.NewStatus(framework.Error, err.Error())
			}
			if err := g.syncSnapshot(); err != nil {
				return framework.NewStatus(framework.Error, err.Error())
			}
		}
	}
	g.rq.free()
	g.rq = newReasonQuery(q, ps)
	kept = true
	res, _, err := g.eng.scheduleOne(g.rq.q, g.rq.pools, seq, false)
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	n := len(g.mir.names)
	words, err := g.eng.filterWords(n)
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	c := &cycle{words: words, chosen: int32(res.node), index: g.mir.index, rq: g.rq}
	if g.prof.RunAllFilters {
		nf := 0 // the profile's device filters (compiler.config's kgpu_config.filters)
		for _, f := range g.prof.Filters {
			if _, ok := filterIDs[f]; ok {
				nf++
			}
		}
		if c.all, err = g.eng.filterWordsAll(nf, n); err != nil {
			return framework.NewStatus(framework.Error, err.Error())
		}
	}
	if g.prof.Mode == "shadow" {
		// every replaced score plugin's normalized (unweighted) value per node: the shadow plugins
		// return them, the framework weights and sums them (framework.go:632-648)
		c.norm = make(map[int32][]int64, len(g.prof.Scores))
		for _, s := range g.prof.Scores {
			id := scoreIDs[s.Name]
			_, norm, err := g.eng.scores(int(id), n)
			if err != nil {
				return framework.NewStatus(framework.Error, err.Error())
			}
			c.norm[id] = norm
		}
	}
	cs.Write(stateKey, c)
	return nil
}

func (g *GpuEval) PreFilterExtensions() framework.PreFilterExtensions { return nil }

// Filter: O(1) lookup of the node's status word.  With nominated pods the framework calls Filter
// twice per node (podPassesFiltersOnNode); the word already combines both passes, and returning it
// for either call yields the framework's verdict and status.
func (g *GpuEval) Filter(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) *framework.Status {
	c, err := readCycle(cs)
	if err != nil {
		return framework.NewStatus(framework.Error, err.Error())
	}
	if c.words == nil { // a batch-served cycle: the chosen node passes, the framework takes it unscored
		if c.index[ni.Node().Name] == c.chosen {
			return nil
		}
		return framework.NewStatus(framework.Unschedulable, "node(s) were not chosen by the batched cycle")
	}
	i := g.mir.index[ni.Node().Name]
	w := c.words[i]
	if w == 0 || w == C.KGPU_FS_NOT_EVALUATED {
		return nil
	}
	if c.all == nil {
		rs, err := g.filterReasons(c.rq, i, w, ni.Node())
		if err != nil {
			return framework.NewStatus(framework.Error, err.Error())
		}
		return framework.NewStatus(framework.Code((w>>8)&3), rs...)
	}
	// runAllFilters: PluginToStatus.Merge (interface.go:162-191) of every failing plugin's status --
	// the merged code is w's, the reasons every failing plugin's in profile order
	n := len(c.words)
	var rs []string
	for p := 0; p*n < len(c.all); p++ {
		if wp := c.all[p*n+int(i)]; wp != 0 {
			r, err := g.filterReasons(c.rq, i, wp, ni.Node())
			if err != nil {
				return framework.NewStatus(framework.Error, err.Error())
			}
			rs = append(rs, r...)
		}
	}
	return framework.NewStatus(framework.Code((w>>8)&3), rs...)
}

func (g *GpuEval) Score(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	c, err := readCycle(cs)
	if err != nil {
		return 0, framework.NewStatus(framework.Error, err.Error())
	}
	i, ok := c.index[node]
	if !ok {
		return 0, framework.NewStatus(framework.Error, fmt.Sprintf("node %q is not in the device mirror", node))
	}
	if i == c.chosen {
		return framework.MaxNodeScore, nil
	}
	return 0, nil
}

func (g *GpuEval) ScoreExtensions() framework.ScoreExtensions { return nil }

// Reserve / Unreserve: cache.AssumePod (scheduler.go:586-593, right after Reserve) / ForgetPod change
// the NodeInfo; the next PreFilter's generation diff carries it to the device.  The node is marked so
// that diff looks at it (track.go).
func (g *GpuEval) Reserve(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, node string) *framework.Status {
	g.track.mark(node)
	if pod.UID == g.lastPod {
		g.lastRes = true
	}
	return nil
}
func (g *GpuEval) Unreserve(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, node string) {
	g.track.mark(node)
	g.track.requeue(pod.UID) // the error func re-queues it (scheduler.go recordSchedulingFailure)
}

// Close releases the plugin: it leaves the ForFramework registry (which otherwise keeps it, and its
// device context, alive for the life of the process) and destroys its engine.  Call it when the
// scheduler that built the profile is torn down or rebuilt.
func (g *GpuEval) Close() {
	unregister(g)
	g.rq.free()
	g.rq = nil
	if g.eng != nil {
		g.eng.close()
		g.eng = nil
	}
	g.mir = nil
	g.comp.close()
	g.comp = nil
}

// New is the framework.PluginFactory (registry.go:28).
func New(obj runtime.Object, h framework.FrameworkHandle) (framework.Plugin, error) {
	prof, err := argsFrom(obj)
	if err != nil {
		return nil, err
	}
	g := &GpuEval{h: h, prof: prof, track: newTracker(), exact: prof.ExactSync}
	if prof.BatchAhead > 1 && prof.Mode != "shadow" {
		g.ahead = &ahead{depth: prof.BatchAhead}
	}
	g.watch()
	register(h, g) // genericScheduler.Preempt finds it by the profile's framework (preempt.go)
	return g, nil
}

// defaultSelector: helper.DefaultSelector (helper/spread.go:29-72) from the handle's listers.
func (g *GpuEval) defaultSelector(pod *v1.Pod) *metav1LabelSelector {
	return defaultSelectorFromListers(g.h, pod)
}
