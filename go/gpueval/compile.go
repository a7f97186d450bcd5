package gpueval

// The PreFilter-time host work (mirror of kubernetes-1_amd/kgpu/compile.py): strings become
// dictionary ids, selectors become requirement programs over those ids, tolerations become bit
// masks over the cluster's taint dictionary.  The device then compares integers only.

/*
#include "kgpu.h"
*/
import "C"

import (
	"fmt"
	"sort"
	"strconv"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/util/validation"
	v1helper "k8s.io/kubernetes/pkg/apis/core/v1/helper"
	schedutil "k8s.io/kubernetes/pkg/scheduler/util"
	utilnode "k8s.io/kubernetes/pkg/util/node"
)

// strDict assigns dense ids in first-seen order.
type strDict struct {
	ids   map[string]int32
	items []string
}

func newStrDict() *strDict { return &strDict{ids: map[string]int32{}} }

func (d *strDict) add(s string) int32 {
	if i, ok := d.ids[s]; ok {
		return i
	}
	i := int32(len(d.items))
	d.ids[s] = i
	d.items = append(d.items, s)
	return i
}

func (d *strDict) get(s string) int32 {
	if i, ok := d.ids[s]; ok {
		return i
	}
	return -1
}

// keySpace: label keys, each with its own value dictionary (values are topology domains).
type keySpace struct {
	keys *strDict
	vals []*strDict
}

func newKeySpace() *keySpace { return &keySpace{keys: newStrDict()} }

func (k *keySpace) add(key, val string) (int32, int32) {
	ki := k.keys.add(key)
	for int(ki) >= len(k.vals) {
		k.vals = append(k.vals, newStrDict())
	}
	return ki, k.vals[ki].add(val)
}

func (k *keySpace) key(key string) int32 { return k.keys.get(key) }

func (k *keySpace) val(ki int32, v string) int32 {
	if ki < 0 {
		return -1
	}
	return k.vals[ki].get(v)
}

// pools: the variable-length parts kgpu_range fields point into (kgpu_pools).
type pools struct {
	reqs      []C.kgpu_req
	ints      []int32
	words     []uint64
	nodeTerms []C.kgpu_node_term
	prefTerms []C.kgpu_pref_term
	spreads   []C.kgpu_spread
	podTerms  []C.kgpu_pod_term
	scalars   []C.kgpu_scalar_req
	ports     []C.kgpu_port
}

func rng(begin, count int) C.kgpu_range { return C.kgpu_range{begin: C.int32_t(begin), count: C.int32_t(count)} }

func (p *pools) intsRange(xs []int32) C.kgpu_range {
	b := len(p.ints)
	p.ints = append(p.ints, xs...)
	return rng(b, len(xs))
}

func (p *pools) wordsRange(ws []uint64) C.kgpu_range {
	b := len(p.words)
	p.words = append(p.words, ws...)
	return rng(b, len(ws))
}

// toC copies the pools into C memory owned by the arena.
func (p *pools) toC(a *arena) *C.kgpu_pools {
	c := (*C.kgpu_pools)(a.alloc(int(unsafe.Sizeof(C.kgpu_pools{}))))
	c.reqs, c.n_reqs = cReqs(a, p.reqs), C.int32_t(len(p.reqs))
	c.ints, c.n_ints = ci32(a, p.ints), C.int32_t(len(p.ints))
	c.words, c.n_words = cu64(a, p.words), C.int32_t(len(p.words))
	c.node_terms, c.n_node_terms = cNodeTerms(a, p.nodeTerms), C.int32_t(len(p.nodeTerms))
	c.pref_terms, c.n_pref_terms = cPrefTerms(a, p.prefTerms), C.int32_t(len(p.prefTerms))
	c.spreads, c.n_spreads = cSpreads(a, p.spreads), C.int32_t(len(p.spreads))
	c.pod_terms, c.n_pod_terms = cPodTerms(a, p.podTerms), C.int32_t(len(p.podTerms))
	c.scalars, c.n_scalars = cScalars(a, p.scalars), C.int32_t(len(p.scalars))
	c.ports, c.n_ports = cPorts(a, p.ports), C.int32_t(len(p.ports))
	return c
}

type taintKey struct{ key, value, effect string }

// compiler holds the cluster dictionaries of one upload epoch.
type compiler struct {
	prof        *profileArgs
	nkeys, pkeys *keySpace
	ns          *strDict
	taints      map[taintKey]int32
	taintList   []taintKey
	scalars     *strDict
	images      *strDict
	controllers *strDict // kind + "/" + uid
	uids        *strDict // pod UIDs (kgpu_pod_query.uid)
	ips         *strDict
	zones       *strDict
	nodeIndex   map[string]int32
	dims        struct{ S, K, TW int }
}

func newCompiler(prof *profileArgs) *compiler {
	c := &compiler{prof: prof, nkeys: newKeySpace(), pkeys: newKeySpace(), ns: newStrDict(),
		taints: map[taintKey]int32{}, scalars: newStrDict(), images: newStrDict(), controllers: newStrDict(), uids: newStrDict(),
		ips: newStrDict(), zones: newStrDict(), nodeIndex: map[string]int32{}}
	c.ips.add("0.0.0.0")
	for _, r := range prof.scalarResources() {
		c.scalars.add(r)
	}
	return c
}

func (c *compiler) taintID(t taintKey) int32 {
	if i, ok := c.taints[t]; ok {
		return i
	}
	i := int32(len(c.taintList))
	c.taints[t] = i
	c.taintList = append(c.taintList, t)
	return i
}

func (c *compiler) registerNode(n *v1.Node) {
	for k, v := range n.Labels {
		c.nkeys.add(k, v)
	}
	for _, t := range n.Spec.Taints {
		c.taintID(taintKey{t.Key, t.Value, string(t.Effect)})
	}
	for r := range n.Status.Allocatable {
		if v1helper.IsScalarResourceName(r) {
			c.scalars.add(string(r))
		}
	}
	for _, im := range n.Status.Images {
		for _, nm := range im.Names {
			c.images.add(nm)
		}
	}
	if z := utilnode.GetZoneKey(n); z != "" {
		c.zones.add(z)
	}
}

func (c *compiler) registerPod(p *v1.Pod) {
	for k, v := range p.Labels {
		c.pkeys.add(k, v)
	}
	c.ns.add(p.Namespace)
	for _, ctr := range append(append([]v1.Container{}, p.Spec.Containers...), p.Spec.InitContainers...) {
		for r := range ctr.Resources.Requests {
			if v1helper.IsScalarResourceName(r) {
				c.scalars.add(string(r))
			}
		}
	}
}

// ---------------------------------------------------------------- selectors
var labelOps = map[metav1.LabelSelectorOperator]int32{metav1.LabelSelectorOpIn: C.KGPU_OP_IN,
	metav1.LabelSelectorOpNotIn: C.KGPU_OP_NOTIN, metav1.LabelSelectorOpExists: C.KGPU_OP_EXISTS,
	metav1.LabelSelectorOpDoesNotExist: C.KGPU_OP_DNE}

// req compiles one requirement; values no object carries are dropped (they can match nothing).
func (c *compiler) req(ks *keySpace, p *pools, key string, op int32, vals []string) C.kgpu_req {
	ki := ks.key(key)
	ids := []int32{}
	var imm int64
	for _, v := range vals {
		if vi := ks.val(ki, v); vi >= 0 {
			ids = append(ids, vi)
		}
	}
	if op == C.KGPU_OP_GT || op == C.KGPU_OP_LT {
		imm, _ = strconv.ParseInt(vals[0], 10, 64)
	}
	return C.kgpu_req{key: C.int32_t(ki), op: C.int32_t(op), vals: p.intsRange(ids), imm: C.int64_t(imm)}
}

// labelSelector: metav1.LabelSelectorAsSelector (nil -> Nothing, empty -> Everything).
func (c *compiler) labelSelector(p *pools, ls *metav1.LabelSelector) (C.kgpu_selector, error) {
	if ls == nil {
		return C.kgpu_selector{kind: C.KGPU_SEL_NOTHING}, nil
	}
	b := len(p.reqs)
	keys := make([]string, 0, len(ls.MatchLabels))
	for k := range ls.MatchLabels {
		keys = append(keys, k)
	}
	sort.Strings(keys)
	for _, k := range keys {
		if errs := validation.IsQualifiedName(k); len(errs) > 0 {
			return C.kgpu_selector{}, fmt.Errorf("invalid label key %q", k)
		}
		p.reqs = append(p.reqs, c.req(c.pkeys, p, k, C.KGPU_OP_IN, []string{ls.MatchLabels[k]}))
	}
	for _, e := range ls.MatchExpressions {
		op, ok := labelOps[e.Operator]
		if !ok {
			return C.kgpu_selector{}, fmt.Errorf("%q is not a valid pod selector operator", e.Operator)
		}
		p.reqs = append(p.reqs, c.req(c.pkeys, p, e.Key, op, e.Values))
	}
	return C.kgpu_selector{kind: C.KGPU_SEL_AND, reqs: rng(b, len(p.reqs)-b)}, nil
}

// nodeTerm: a required NodeSelectorTerm (helpers.go:317-346).
func (c *compiler) nodeTerm(p *pools, t v1.NodeSelectorTerm) C.kgpu_node_term {
	out := C.kgpu_node_term{field_op: -1, field_node: -1}
	if len(t.MatchExpressions) == 0 && len(t.MatchFields) == 0 {
		out.never_match = 1
		return out
	}
	b := len(p.reqs)
	for _, e := range t.MatchExpressions {
		var op int32
		switch e.Operator {
		case v1.NodeSelectorOpIn:
			op = C.KGPU_OP_IN
		case v1.NodeSelectorOpNotIn:
			op = C.KGPU_OP_NOTIN
		case v1.NodeSelectorOpExists:
			op = C.KGPU_OP_EXISTS
		case v1.NodeSelectorOpDoesNotExist:
			op = C.KGPU_OP_DNE
		case v1.NodeSelectorOpGt:
			op = C.KGPU_OP_GT
		case v1.NodeSelectorOpLt:
			op = C.KGPU_OP_LT
		default:
			out.never_match = 1
			return out
		}
		p.reqs = append(p.reqs, c.req(c.nkeys, p, e.Key, op, e.Values))
	}
	out.reqs = rng(b, len(p.reqs)-b)
	for _, f := range t.MatchFields {
		if f.Key != "metadata.name" || len(f.Values) != 1 {
			out.never_match = 1
			continue
		}
		if f.Operator == v1.NodeSelectorOpIn {
			out.field_op = C.KGPU_OP_IN
		} else {
			out.field_op = C.KGPU_OP_NOTIN
		}
		if i, ok := c.nodeIndex[f.Values[0]]; ok {
			out.field_node = C.int32_t(i)
		}
	}
	return out
}

// ---------------------------------------------------------------- resources
// podRequest: computePodResourceRequest (noderesources/fit.go:112-129): containers summed, init
// containers as a max, overhead added.
func podRequest(p *v1.Pod) (cpu, mem, eph int64, scalars map[string]int64) {
	scalars = map[string]int64{}
	add := func(rl v1.ResourceList, max bool) {
		for r, q := range rl {
			var cur *int64
			v := q.Value()
			switch r {
			case v1.ResourceCPU:
				cur, v = &cpu, q.MilliValue()
			case v1.ResourceMemory:
				cur = &mem
			case v1.ResourceEphemeralStorage:
				cur = &eph
			default:
				if !v1helper.IsScalarResourceName(r) {
					continue
				}
				x := scalars[string(r)]
				cur = &x
				defer func(name string) { scalars[name] = x }(string(r))
			}
			if max {
				if v > *cur {
					*cur = v
				}
			} else {
				*cur += v
			}
		}
	}
	for _, ctr := range p.Spec.Containers {
		add(ctr.Resources.Requests, false)
	}
	for _, ctr := range p.Spec.InitContainers {
		add(ctr.Resources.Requests, true)
	}
	if p.Spec.Overhead != nil {
		add(p.Spec.Overhead, false)
	}
	return
}

// scoreRequest: calculatePodResourceRequest (resource_allocation.go:118-142) with the non-zero
// defaults of schedutil.GetNonzeroRequestForResource.
func scoreRequest(p *v1.Pod, r v1.ResourceName) int64 {
	var v int64
	for i := range p.Spec.Containers {
		v += schedutil.GetNonzeroRequestForResource(r, &p.Spec.Containers[i].Resources.Requests)
	}
	for i := range p.Spec.InitContainers {
		if x := schedutil.GetNonzeroRequestForResource(r, &p.Spec.InitContainers[i].Resources.Requests); x > v {
			v = x
		}
	}
	if p.Spec.Overhead != nil {
		if q, ok := p.Spec.Overhead[r]; ok {
			v += q.Value()
		}
	}
	return v
}

// scalarNames: a pod's scalar requests in query order (kgpu_pod_query.scalars; the names
// kgpu_filter_reasons quotes in "Insufficient <name>").
func scalarNames(sc map[string]int64) []string {
	names := make([]string, 0, len(sc))
	for r := range sc {
		names = append(names, r)
	}
	sort.Strings(names)
	return names
}

// ---------------------------------------------------------------- pod query
func toleratesTaint(t v1.Toleration, k taintKey) bool {
	tt := v1.Taint{Key: k.key, Value: k.value, Effect: v1.TaintEffect(k.effect)}
	return t.ToleratesTaint(&tt)
}

// compilePod builds the kgpu_pod_query of a pod (the PreFilter-time state of every replaced
// plugin).  Mirrors kubernetes-1_amd/kgpu/compile.py Compiler.compile_pod.
func (c *compiler) compilePod(pod *v1.Pod, p *pools) (C.kgpu_pod_query, error) {
	var q C.kgpu_pod_query
	var flags uint32
	q.ns = C.int32_t(c.ns.add(pod.Namespace))
	cpu, mem, eph, sc := podRequest(pod)
	q.req[0], q.req[1], q.req[2] = C.int64_t(cpu), C.int64_t(mem), C.int64_t(eph)
	q.score_req[0] = C.int64_t(scoreRequest(pod, v1.ResourceCPU))
	q.score_req[1] = C.int64_t(scoreRequest(pod, v1.ResourceMemory))
	q.score_req[2] = C.int64_t(scoreRequest(pod, v1.ResourceEphemeralStorage))
	// NonZeroRequested delta of NodeInfo.AddPod (types.go:524-555): the same non-zero defaults
	q.nz[0], q.nz[1] = q.score_req[0], q.score_req[1]
	if cpu == 0 && mem == 0 && eph == 0 && len(sc) == 0 {
		flags |= C.KGPU_Q_FIT_ALL_ZERO
	}
	names := scalarNames(sc)
	b := len(p.scalars)
	for _, r := range names {
		col := c.scalars.get(r)
		_, ignored := c.prof.ignoredResources[r]
		check := C.int32_t(1)
		if ignored {
			check = 0
		}
		p.scalars = append(p.scalars, C.kgpu_scalar_req{col: C.int32_t(col), check: check, value: C.int64_t(sc[r]),
			score_value: C.int64_t(scoreRequest(pod, v1.ResourceName(r)))})
	}
	q.scalars = rng(b, len(p.scalars)-b)
	q.node_name = -1
	if pod.Spec.NodeName != "" {
		q.node_name = -2
		if i, ok := c.nodeIndex[pod.Spec.NodeName]; ok {
			q.node_name = C.int32_t(i)
		}
	}
	q.n_containers = C.int32_t(len(pod.Spec.Containers))
	// host ports (types.go:728-731)
	b = len(p.ports)
	for _, ctr := range pod.Spec.Containers {
		for _, pt := range ctr.Ports {
			if pt.HostPort <= 0 {
				continue
			}
			ip := pt.HostIP
			if ip == "" {
				ip = "0.0.0.0"
			}
			proto := map[v1.Protocol]int32{v1.ProtocolTCP: 0, v1.ProtocolUDP: 1, v1.ProtocolSCTP: 2, "": 0}[pt.Protocol]
			p.ports = append(p.ports, C.kgpu_port{ip: C.int32_t(c.ips.add(ip)), proto: C.int32_t(proto), port: C.int32_t(pt.HostPort)})
		}
	}
	q.ports = rng(b, len(p.ports)-b)
	// tolerations as masks over the taint dictionary (taint_toleration.go:54-152)
	TW := c.dims.TW
	nosched, prefer := make([]uint64, TW), make([]uint64, TW)
	for id, k := range c.taintList {
		if id/64 >= TW {
			break
		}
		for _, t := range pod.Spec.Tolerations {
			if !toleratesTaint(t, k) {
				continue
			}
			if k.effect == string(v1.TaintEffectPreferNoSchedule) {
				if t.Effect == "" || t.Effect == v1.TaintEffectPreferNoSchedule {
					prefer[id/64] |= 1 << (uint(id) % 64)
				}
			} else {
				nosched[id/64] |= 1 << (uint(id) % 64)
			}
		}
	}
	q.tol_nosched, q.tol_prefer = p.wordsRange(nosched), p.wordsRange(prefer)
	for _, t := range pod.Spec.Tolerations {
		if toleratesTaint(t, taintKey{v1.TaintNodeUnschedulable, "", string(v1.TaintEffectNoSchedule)}) {
			flags |= C.KGPU_Q_TOLERATES_UNSCHEDULABLE
		}
	}
	// nodeSelector + required / preferred node affinity (node_affinity.go, helpers.go)
	b = len(p.reqs)
	for k, v := range pod.Spec.NodeSelector {
		p.reqs = append(p.reqs, c.req(c.nkeys, p, k, C.KGPU_OP_IN, []string{v}))
	}
	q.node_selector = rng(b, len(p.reqs)-b)
	if a := pod.Spec.Affinity; a != nil && a.NodeAffinity != nil {
		if r := a.NodeAffinity.RequiredDuringSchedulingIgnoredDuringExecution; r != nil {
			flags |= C.KGPU_Q_REQ_NODE_AFFINITY
			b = len(p.nodeTerms)
			for _, t := range r.NodeSelectorTerms {
				p.nodeTerms = append(p.nodeTerms, c.nodeTerm(p, t))
			}
			q.req_terms = rng(b, len(p.nodeTerms)-b)
		}
		b = len(p.prefTerms)
		for _, t := range a.NodeAffinity.PreferredDuringSchedulingIgnoredDuringExecution {
			nt := c.nodeTerm(p, t.Preference)
			sel := C.kgpu_selector{kind: C.KGPU_SEL_AND, reqs: nt.reqs}
			if nt.never_match != 0 {
				sel.kind = C.KGPU_SEL_NOTHING
			}
			p.prefTerms = append(p.prefTerms, C.kgpu_pref_term{weight: C.int32_t(t.Weight), sel: sel})
		}
		q.pref_terms = rng(b, len(p.prefTerms)-b)
	}
	// ImageLocality (image_locality.go:84-98): normalized image ids per container
	ims := make([]int32, 0, len(pod.Spec.Containers))
	known := false
	for _, ctr := range pod.Spec.Containers {
		id := c.images.get(normalizedImageName(ctr.Image))
		known = known || id >= 0
		ims = append(ims, id)
	}
	q.images = p.intsRange(ims)
	if !known {
		flags |= C.KGPU_Q_NO_KNOWN_IMAGE
	}
	// NodePreferAvoidPods: controllerRef of kind ReplicationController / ReplicaSet
	q.avoid_id = -1
	if ref := metav1.GetControllerOf(pod); ref != nil && (ref.Kind == "ReplicationController" || ref.Kind == "ReplicaSet") {
		q.avoid_id = C.int32_t(c.controllers.get(ref.Kind + "/" + string(ref.UID)))
	}
	// PodTopologySpread constraints (podtopologyspread/common.go:34-72)
	if len(pod.Spec.TopologySpreadConstraints) > 0 {
		flags |= C.KGPU_Q_HAS_TSC
	}
	var err error
	if q.pts_hard, err = c.spreads(pod, p, v1.DoNotSchedule); err != nil {
		return q, err
	}
	if q.pts_soft, err = c.spreads(pod, p, v1.ScheduleAnyway); err != nil {
		return q, err
	}
	q.dpts = C.kgpu_selector{kind: C.KGPU_SEL_EMPTY} // DefaultSelector: set by the plugin from its listers
	// InterPodAffinity terms (types.go:92-160)
	if a := pod.Spec.Affinity; a != nil {
		if a.PodAffinity != nil {
			flags |= C.KGPU_Q_HAS_POD_AFFINITY
			q.ipa_req_aff = c.podTerms(pod, p, a.PodAffinity.RequiredDuringSchedulingIgnoredDuringExecution, nil)
			q.ipa_pref_aff = c.podTerms(pod, p, nil, a.PodAffinity.PreferredDuringSchedulingIgnoredDuringExecution)
		}
		if a.PodAntiAffinity != nil {
			flags |= C.KGPU_Q_HAS_POD_ANTI
			q.ipa_req_anti = c.podTerms(pod, p, a.PodAntiAffinity.RequiredDuringSchedulingIgnoredDuringExecution, nil)
			q.ipa_pref_anti = c.podTerms(pod, p, nil, a.PodAntiAffinity.PreferredDuringSchedulingIgnoredDuringExecution)
		}
	}
	keys := make([]string, 0, len(pod.Labels))
	for k := range pod.Labels {
		keys = append(keys, k)
	}
	sort.Strings(keys)
	pairs := make([]int32, 0, 2*len(keys))
	for _, k := range keys {
		ki, vi := c.pkeys.add(k, pod.Labels[k])
		pairs = append(pairs, ki, vi)
	}
	q.labels = p.intsRange(pairs)
	if pod.DeletionTimestamp != nil {
		flags |= C.KGPU_Q_TERMINATING
	}
	// NodeResourceLimits (resource_limits.go:145-156)
	var lc, lm int64
	for _, ctr := range pod.Spec.Containers {
		lc += ctr.Resources.Limits.Cpu().MilliValue()
		lm += ctr.Resources.Limits.Memory().Value()
	}
	for _, ctr := range pod.Spec.InitContainers {
		if x := ctr.Resources.Limits.Cpu().MilliValue(); x > lc {
			lc = x
		}
		if x := ctr.Resources.Limits.Memory().Value(); x > lm {
			lm = x
		}
	}
	q.limits[0], q.limits[1] = C.int64_t(lc), C.int64_t(lm)
	if pod.Spec.Priority != nil { // podutil.GetPodPriority
		q.priority = C.int32_t(*pod.Spec.Priority)
	}
	q.uid = C.int64_t(c.uids.add(string(pod.UID)) + 1) // addNominatedPods skips the pod itself by UID
	q.flags = C.uint32_t(flags)
	return q, nil
}

func (c *compiler) spreads(pod *v1.Pod, p *pools, action v1.UnsatisfiableConstraintAction) (C.kgpu_range, error) {
	b := len(p.spreads)
	for _, tsc := range pod.Spec.TopologySpreadConstraints {
		if tsc.WhenUnsatisfiable != action {
			continue
		}
		sel, err := c.labelSelector(p, tsc.LabelSelector)
		if err != nil {
			return rng(0, 0), err
		}
		self := int32(0)
		if s, err := metav1.LabelSelectorAsSelector(tsc.LabelSelector); err == nil && s.Matches(labelsSet(pod.Labels)) {
			self = 1
		}
		host := int32(0)
		if tsc.TopologyKey == v1.LabelHostname {
			host = 1
		}
		p.spreads = append(p.spreads, C.kgpu_spread{max_skew: C.int32_t(tsc.MaxSkew), key: C.int32_t(c.nkeys.key(tsc.TopologyKey)),
			is_hostname: C.int32_t(host), self_match: C.int32_t(self), sel: sel})
	}
	return rng(b, len(p.spreads)-b), nil
}

func (c *compiler) podTerms(pod *v1.Pod, p *pools, req []v1.PodAffinityTerm, pref []v1.WeightedPodAffinityTerm) C.kgpu_range {
	b := len(p.podTerms)
	add := func(t v1.PodAffinityTerm, w int32) bool {
		sel, err := c.labelSelector(p, t.LabelSelector)
		if err != nil {
			return false
		}
		nss := t.Namespaces
		if len(nss) == 0 {
			nss = []string{pod.Namespace}
		}
		ids := make([]int32, 0, len(nss))
		for _, n := range nss {
			ids = append(ids, c.ns.add(n))
		}
		p.podTerms = append(p.podTerms, C.kgpu_pod_term{weight: C.int32_t(w), topo_key: C.int32_t(c.nkeys.key(t.TopologyKey)),
			ns: p.intsRange(ids), sel: sel})
		return true
	}
	for _, t := range req {
		if !add(t, 0) { // getAffinityTerms: one invalid selector drops the list
			p.podTerms = p.podTerms[:b]
			return rng(b, 0)
		}
	}
	for _, t := range pref {
		if !add(t.PodAffinityTerm, t.Weight) {
			p.podTerms = p.podTerms[:b]
			return rng(b, 0)
		}
	}
	return rng(b, len(p.podTerms)-b)
}

func normalizedImageName(name string) string {
	lc, ls := -1, -1
	for i := 0; i < len(name); i++ {
		switch name[i] {
		case ':':
			lc = i
		case '/':
			ls = i
		}
	}
	if lc <= ls {
		name += ":latest"
	}
	return name
}
