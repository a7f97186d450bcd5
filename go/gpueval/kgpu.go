// Package gpueval is the out-of-tree plugin set that runs kube-scheduler's per-pod node
// evaluation on an MI355X through libkgpu.so (include/kgpu.h).  Register it with
// app.WithPlugin(gpueval.Name, gpueval.New) (cmd/kube-scheduler/app/server.go:302-307).
//
// This file is the cgo binding: one method per C entry point.  All buffers handed to C are C
// memory (cgo forbids passing Go memory that holds Go pointers), owned by an arena that the
// caller frees after the call.
package gpueval

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../kubernetes-1_amd/kgpu -lkgpu -Wl,-rpath,${SRCDIR}/../../kubernetes-1_amd/kgpu
#include <stdlib.h>
#include <string.h>
#include "kgpu.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

// arena owns C allocations made for one call, and the C objects (pool sets) that must outlive it.
type arena struct {
	ptrs []unsafe.Pointer
	fns  []func()
}

// onFree runs f when the arena is freed (after its memory is released).
func (a *arena) onFree(f func()) { a.fns = append(a.fns, f) }

func (a *arena) alloc(bytes int) unsafe.Pointer {
	if bytes <= 0 {
		bytes = 1
	}
	p := C.calloc(1, C.size_t(bytes))
	a.ptrs = append(a.ptrs, p)
	return p
}

func (a *arena) free() {
	for _, p := range a.ptrs {
		C.free(p)
	}
	a.ptrs = nil
	for _, f := range a.fns {
		f()
	}
	a.fns = nil
}

// cmem copies n elements of elem bytes from a Go slice of plain values (no Go pointers inside)
// into C memory owned by the arena.  The typed wrappers below replace a generic helper: the
// reference tree builds with go 1.13 (/root/reference/go.mod), which has no type parameters.
func cmem(a *arena, first unsafe.Pointer, n, elem int) unsafe.Pointer {
	p := a.alloc(n * elem)
	C.memcpy(p, first, C.size_t(n*elem))
	return p
}

func ci32(a *arena, s []int32) *C.int32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int32_t)(cmem(a, unsafe.Pointer(&s[0]), len(s), 4))
}

func ci64(a *arena, s []int64) *C.int64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int64_t)(cmem(a, unsafe.Pointer(&s[0]), len(s), 8))
}

func cu8(a *arena, s []uint8) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(cmem(a, unsafe.Pointer(&s[0]), len(s), 1))
}











func cQueries(a *arena, s []C.kgpu_pod_query) *C.kgpu_pod_query {
	if len(s) == 0 {
		return nil
	}
	return (*C.kgpu_pod_query)(cmem(a, unsafe.Pointer(&s[0]), len(s), int(unsafe.Sizeof(s[0]))))
}

func cNominated(a *arena, s []C.kgpu_nominated) *C.kgpu_nominated {
	if len(s) == 0 {
		return nil
	}
	return (*C.kgpu_nominated)(cmem(a, unsafe.Pointer(&s[0]), len(s), int(unsafe.Sizeof(s[0]))))
}

func cVictims(a *arena, s []C.kgpu_victim) *C.kgpu_victim {
	if len(s) == 0 {
		return nil
	}
	return (*C.kgpu_victim)(cmem(a, unsafe.Pointer(&s[0]), len(s), int(unsafe.Sizeof(s[0]))))
}

func cDeltas(a *arena, s []C.kgpu_delta) *C.kgpu_delta {
	if len(s) == 0 {
		return nil
	}
	return (*C.kgpu_delta)(cmem(a, unsafe.Pointer(&s[0]), len(s), int(unsafe.Sizeof(s[0]))))
}

func cNodeRows(a *arena, s []C.kgpu_node_row) *C.kgpu_node_row {
	if len(s) == 0 {
		return nil
	}
	return (*C.kgpu_node_row)(cmem(a, unsafe.Pointer(&s[0]), len(s), int(unsafe.Sizeof(s[0]))))
}

type engine struct{ ctx *C.kgpu_ctx }

func kerr(ctx *C.kgpu_ctx, rc C.int) error {
	if rc == C.KGPU_OK {
		return nil
	}
	msg := "null context"
	if ctx != nil {
		msg = C.GoString(C.kgpu_last_error(ctx))
	}
	return fmt.Errorf("kgpu: %d: %s", int(rc), msg)
}

// newEngine replaces the framework.PluginFactory state of the replaced plugins
// (framework/v1alpha1/registry.go:28) with the profile's plugin list, weights and args
// (framework.go:205-298).
func newEngine(cfg *C.kgpu_config) (*engine, error) {
	if C.kgpu_abi_version() != C.KGPU_ABI_VERSION {
		return nil, fmt.Errorf("kgpu: ABI version mismatch")
	}
	var ctx *C.kgpu_ctx
	if rc := C.kgpu_create(cfg, &ctx); rc != C.KGPU_OK {
		return nil, fmt.Errorf("kgpu_create: %d", int(rc))
	}
	return &engine{ctx: ctx}, nil
}

// uploadSnapshot mirrors cache.UpdateSnapshot (internal/cache/cache.go:202-301) from scratch.
func (e *engine) uploadSnapshot(s *C.kgpu_snapshot, generation int64) error {
	return kerr(e.ctx, C.kgpu_upload_snapshot(e.ctx, s, C.int64_t(generation)))
}

// applyDelta sends the NodeInfo changes since the last sync (kgpu_apply_delta): AddPod /
// RemovePod by UID, SetNode, and the Snapshot.List() rebuild after node adds / removes.
func (e *engine) applyDelta(b *C.kgpu_delta_batch, generation int64) ([]int32, error) {
	n := int(b.n_deltas)
	slots := make([]int32, n+1)
	rc := C.kgpu_apply_delta(e.ctx, b, C.int64_t(generation), (*C.int32_t)(unsafe.Pointer(&slots[0])))
	return slots[:n], kerr(e.ctx, rc)
}

// scheduleOne is genericScheduler.Schedule (core/generic_scheduler.go:146-209) for one pod: the
// filter statuses, scores and the selected node stay on the device for the lookups below.
func (e *engine) scheduleOne(q *C.kgpu_pod_query, pools *C.kgpu_pools, seq int64, assume bool) (C.kgpu_result, int32, error) {
	var res C.kgpu_result
	var slot C.int32_t
	a := C.int32_t(0)
	if assume {
		a = 1
	}
	rc := C.kgpu_schedule_one(e.ctx, q, pools, C.int64_t(seq), a, &res, &slot)
	return res, int32(slot), kerr(e.ctx, rc)
}

// scheduleBatch is the scheduleOne loop (scheduler.go:509-593) over queued pods with on-device
// assume: the throughput path.
func (e *engine) scheduleBatch(qs []C.kgpu_pod_query, pools *C.kgpu_pools, firstSeq int64) ([]C.kgpu_result, error) {
	if len(qs) == 0 {
		return nil, nil
	}
	var a arena
	defer a.free()
	cq := cQueries(&a, qs)
	res := make([]C.kgpu_result, len(qs))
	var st C.kgpu_stats
	rc := C.kgpu_schedule_batch(e.ctx, cq, C.int32_t(len(qs)), pools, C.int64_t(firstSeq),
		(*C.kgpu_result)(unsafe.Pointer(&res[0])), &st)
	return res, kerr(e.ctx, rc)
}

// filterWords copies the per-node PluginToStatus.Merge code words of the last scheduleOne
// (framework.go:477-502): low byte = 1-based position of the first failing filter, bits 8-9 the
// framework.Code, bits 16-31 the plugin detail.
func (e *engine) filterWords(n int) ([]uint32, error) {
	w := make([]uint32, n+1)
	rc := C.kgpu_get_filter(e.ctx, (*C.uint32_t)(unsafe.Pointer(&w[0])))
	return w[:n], kerr(e.ctx, rc)
}

// filterWordsAll copies the last scheduleOne's per-plugin status words under KGPU_OPT_RUN_ALL_FILTERS:
// [filter position][node], each in filterWords' format (0: the plugin passed the node).
func (e *engine) filterWordsAll(nf, n int) ([]uint32, error) {
	w := make([]uint32, nf*n+1)
	rc := C.kgpu_get_filter_all(e.ctx, (*C.uint32_t)(unsafe.Pointer(&w[0])))
	return w[:nf*n], kerr(e.ctx, rc)
}

// setOption is kgpu_set_option.
func (e *engine) setOption(opt C.int32_t, v int64) error {
	return kerr(e.ctx, C.kgpu_set_option(e.ctx, opt, C.int64_t(v)))
}

// scores returns one score plugin's raw and normalized (unweighted) values per node.
func (e *engine) scores(plugin int, n int) (raw, norm []int64, err error) {
	raw, norm = make([]int64, n+1), make([]int64, n+1)
	rc := C.kgpu_get_scores(e.ctx, C.int32_t(plugin), (*C.int64_t)(unsafe.Pointer(&raw[0])),
		(*C.int64_t)(unsafe.Pointer(&norm[0])))
	return raw[:n], norm[:n], kerr(e.ctx, rc)
}

// preparePods registers the topology pod classes of pods expected soon (kgpu_prepare_pods): their count
// columns are filled now, not on the cycle of the first pod that needs them.
func (e *engine) preparePods(qs []C.kgpu_pod_query, pools *C.kgpu_pools) error {
	if len(qs) == 0 {
		return nil
	}
	var a arena
	defer a.free()
	return kerr(e.ctx, C.kgpu_prepare_pods(e.ctx, cQueries(&a, qs), C.int32_t(len(qs)), pools))
}

func (e *engine) forget(slot int32) error { return kerr(e.ctx, C.kgpu_forget_pod(e.ctx, C.int32_t(slot))) }
func (e *engine) generation() int64       { return int64(C.kgpu_generation(e.ctx)) }
func (e *engine) close()                  { C.kgpu_destroy(e.ctx) }

// Node sharding across the GPUs of one host (SURVEY.md 8(e)): one engine per GPU holding a
// contiguous slice of Snapshot.List() (kgpu_snapshot.node_base / n_total_nodes).  Rank 0 creates
// the RCCL id; every engine then receives the same calls with the same arguments, in order.
func commUniqueID() ([128]byte, error) {
	var id [128]byte
	rc := C.kgpu_comm_unique_id((*C.uint8_t)(unsafe.Pointer(&id[0])))
	return id, kerr(nil, rc)
}

func (e *engine) commInit(nranks, rank int, id [128]byte) error {
	return kerr(e.ctx, C.kgpu_comm_init(e.ctx, C.int32_t(nranks), C.int32_t(rank), (*C.uint8_t)(unsafe.Pointer(&id[0]))))
}

// setNominated replaces the engine's copy of the PodNominator (kgpu_set_nominated): while it is
// non-empty every cycle runs podPassesFiltersOnNode's two passes (generic_scheduler.go:526-615).
func (e *engine) setNominated(noms []C.kgpu_nominated, recs []C.kgpu_pod_query, pools *C.kgpu_pools) error {
	var a arena
	defer a.free()
	var cn *C.kgpu_nominated
	var cr *C.kgpu_pod_query
	if len(noms) > 0 {
		cn, cr = cNominated(&a, noms), cQueries(&a, recs)
	}
	return kerr(e.ctx, C.kgpu_set_nominated(e.ctx, cn, C.int32_t(len(noms)), cr, pools))
}

// selectVictims is selectNodesForPreemption + pickOneNodeForPreemption (generic_scheduler.go:718-1012):
// per-node victims (indices into victims) and the picked node index (-1: none).
func (e *engine) selectVictims(q *C.kgpu_pod_query, pools *C.kgpu_pools, victims []C.kgpu_victim,
	recs []C.kgpu_pod_query, pdbAllowed []int32, n int) ([]C.kgpu_node_victims, []int32, int32, error) {
	var a arena
	defer a.free()
	args := C.kgpu_preempt_args{n_victims: C.int32_t(len(victims)), n_pdbs: C.int32_t(len(pdbAllowed))}
	if len(victims) > 0 {
		args.victims, args.pods = cVictims(&a, victims), cQueries(&a, recs)
	}
	if len(pdbAllowed) > 0 {
		args.pdb_allowed = ci32(&a, pdbAllowed)
	}
	out := make([]C.kgpu_node_victims, n+1)
	vout := make([]int32, len(victims)+1)
	var chosen C.int32_t
	rc := C.kgpu_select_victims(e.ctx, q, pools, &args, &out[0], (*C.int32_t)(unsafe.Pointer(&vout[0])), &chosen)
	return out[:n], vout[:len(victims)], int32(chosen), kerr(e.ctx, rc)
}

// xgmiActive reports whether kgpu_comm_init mapped every peer's mailbox ring: persistent runs then
// exchange their granules over xGMI instead of one RCCL all-gather per pod.
func (e *engine) xgmiActive() bool { return C.kgpu_xgmi_active(e.ctx) != 0 }
