package gpueval

/*
#include "kgpu.h"
*/
import "C"

import (
	"encoding/json"
	"fmt"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/labels"
	"k8s.io/apimachinery/pkg/runtime"
	framework "k8s.io/kubernetes/pkg/scheduler/framework/v1alpha1"
)

type metav1LabelSelector = metav1.LabelSelector

var unsafeSizeofSnapshot = unsafe.Sizeof(C.kgpu_snapshot{})


// argsFrom decodes the GpuEval pluginConfig args (INTEGRATION.md section 4).
func argsFrom(obj runtime.Object) (*profileArgs, error) {
	p := &profileArgs{HardPodAffinityWeight: 1, PercentageOfNodesToScore: 100, Mode: "select", TieBreakSeed: 0x7B,
		LeastResources: map[string]int64{"cpu": 1, "memory": 1}, MostResources: map[string]int64{"cpu": 1, "memory": 1},
		ignoredResources: map[string]struct{}{}}
	if u, ok := obj.(*runtime.Unknown); ok && u != nil && len(u.Raw) > 0 {
		if err := json.Unmarshal(u.Raw, p); err != nil {
			return nil, fmt.Errorf("gpueval args: %v", err)
		}
	}
	if len(p.Filters) == 0 && len(p.Scores) == 0 {
		return nil, fmt.Errorf("gpueval args: no filter or score plugins to replace")
	}
	return p, nil
}

// defaultSelectorFromListers: helper.DefaultSelector (helper/spread.go:29-72) as a LabelSelector:
// the selectors of the pod's Services and ReplicationControllers (label sets, merged) and of its
// ReplicaSets and StatefulSets (label selectors, ANDed).  nil: no selector (Empty()).
func defaultSelectorFromListers(h framework.FrameworkHandle, pod *v1.Pod) *metav1.LabelSelector {
	f := h.SharedInformerFactory()
	if f == nil {
		return nil
	}
	set := labels.Set{}
	var exprs []metav1.LabelSelectorRequirement
	podLabels := labels.Set(pod.Labels)
	if svcs, err := f.Core().V1().Services().Lister().Services(pod.Namespace).List(labels.Everything()); err == nil {
		for _, s := range svcs {
			if s.Spec.Selector != nil && labels.SelectorFromSet(s.Spec.Selector).Matches(podLabels) {
				for k, v := range s.Spec.Selector {
					set[k] = v
				}
			}
		}
	}
	if len(pod.Labels) > 0 {
		if rcs, err := f.Core().V1().ReplicationControllers().Lister().ReplicationControllers(pod.Namespace).List(labels.Everything()); err == nil {
			for _, rc := range rcs {
				if rc.Spec.Selector != nil && labels.SelectorFromSet(rc.Spec.Selector).Matches(podLabels) {
					for k, v := range rc.Spec.Selector {
						set[k] = v
					}
				}
			}
		}
		if rss, err := f.Apps().V1().ReplicaSets().Lister().ReplicaSets(pod.Namespace).List(labels.Everything()); err == nil {
			for _, rs := range rss {
				if sel, err := metav1.LabelSelectorAsSelector(rs.Spec.Selector); err == nil && sel.Matches(podLabels) {
					exprs = append(exprs, toExprs(rs.Spec.Selector)...)
				}
			}
		}
		if sss, err := f.Apps().V1().StatefulSets().Lister().StatefulSets(pod.Namespace).List(labels.Everything()); err == nil {
			for _, ss := range sss {
				if sel, err := metav1.LabelSelectorAsSelector(ss.Spec.Selector); err == nil && sel.Matches(podLabels) {
					exprs = append(exprs, toExprs(ss.Spec.Selector)...)
				}
			}
		}
	}
	if len(set) == 0 && len(exprs) == 0 {
		return nil
	}
	return &metav1.LabelSelector{MatchLabels: set, MatchExpressions: exprs}
}

func toExprs(ls *metav1.LabelSelector) []metav1.LabelSelectorRequirement {
	if ls == nil {
		return nil
	}
	out := append([]metav1.LabelSelectorRequirement{}, ls.MatchExpressions...)
	for k, v := range ls.MatchLabels {
		out = append(out, metav1.LabelSelectorRequirement{Key: k, Operator: metav1.LabelSelectorOpIn, Values: []string{v}})
	}
	return out
}

// reasonQuery is the C copy of one cycle's pod query, its pool set and its scalar request names,
// kept from PreFilter until the next PreFilter so that Filter can have its status reasons formatted.
type reasonQuery struct {
	a     arena
	ps    *poolSet
	q     *C.kgpu_pod_query
	pools *C.kgpu_pools
	names **C.char
}

// newReasonQuery takes ownership of ps (the set q was compiled into).
func newReasonQuery(q C.kgpu_pod_query, ps *poolSet) *reasonQuery {
	r := &reasonQuery{ps: ps}
	r.q = cQueries(&r.a, []C.kgpu_pod_query{q})
	r.pools = ps.toC(&r.a)
	// the names of the pod's scalar requests, in query order (what "Insufficient <name>" quotes)
	if n := int(q.scalars.count); n > 0 {
		arr := (*[1 << 20]*C.char)(r.a.alloc(n * int(unsafe.Sizeof((*C.char)(nil)))))
		for i := 0; i < n; i++ {
			cs := C.CString(ps.scalarName(int32(q.scalars.begin) + int32(i)))
			r.a.ptrs = append(r.a.ptrs, unsafe.Pointer(cs))
			arr[i] = cs
		}
		r.names = &arr[0]
	}
	return r
}

func (r *reasonQuery) free() {
	if r != nil {
		r.a.free()
		r.ps.free()
	}
}

// filterReasons: the failing plugin's status reasons for node `node`'s status word, formatted by
// kgpu_filter_reasons -- the formatter the Python mirror calls too (kgpu/framework.py
// status_reasons), pinned by the reference's filter tables under -m gpu.  The node's Spec.Taints
// go in spec order with their dictionary ids (TaintToleration names the first untolerated one,
// taint_toleration.go:59-71).
func (g *GpuEval) filterReasons(rq *reasonQuery, node int32, w uint32, n *v1.Node) ([]string, error) {
	if rq == nil {
		return nil, fmt.Errorf("gpueval: no compiled query for this cycle's status reasons")
	}
	var a arena
	defer a.free()
	var args C.kgpu_reason_args
	args.q, args.pools, args.node, args.word = rq.q, rq.pools, C.int32_t(node), C.uint32_t(w)
	args.scalar_names = rq.names
	if n != nil && len(n.Spec.Taints) > 0 {
		tr := (*[1 << 20]C.kgpu_taint_ref)(a.alloc(len(n.Spec.Taints) * int(unsafe.Sizeof(C.kgpu_taint_ref{}))))
		for i, t := range n.Spec.Taints {
			id := g.comp.taintID(t) // -1: not in the dictionary
			k, v, e := C.CString(t.Key), C.CString(t.Value), C.CString(string(t.Effect))
			a.ptrs = append(a.ptrs, unsafe.Pointer(k), unsafe.Pointer(v), unsafe.Pointer(e))
			tr[i] = C.kgpu_taint_ref{key: k, value: v, effect: e, id: C.int32_t(id)}
		}
		args.taints, args.n_taints = &tr[0], C.int32_t(len(n.Spec.Taints))
	}
	buf := make([]byte, 512)
	for {
		var need C.int64_t
		cb := a.alloc(len(buf))
		rc := C.kgpu_filter_reasons(g.eng.ctx, &args, (*C.char)(cb), C.int64_t(len(buf)), &need)
		if rc == C.KGPU_E_CAPACITY {
			buf = make([]byte, int(need))
			continue
		}
		if rc < 0 {
			return nil, kerr(g.eng.ctx, rc)
		}
		raw := C.GoBytes(cb, C.int(need))
		out := make([]string, 0, int(rc))
		for start, i := 0, 0; i < len(raw) && len(out) < int(rc); i++ {
			if raw[i] == 0 {
				out = append(out, string(raw[start:i]))
				start = i + 1
			}
		}
		return out, nil
	}
}
