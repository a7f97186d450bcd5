// kgpu_staging.h -- the host-side staging bookkeeping of libkgpu, free of HIP.
//
// kgpu_api.cpp moves every host-to-device copy of a call out of a few pinned blocks (the query
// pools, a topology run's tables, a delta batch, the short-cycle arena) so that each call pays one
// or two stream operations.  The copies are asynchronous: a block may be read by a pending copy long
// after the call that filled it returned (an error exit skips the final synchronize).  The rule this
// file enforces is the one the round-3 use-after-free broke (a pinned staging block freed when
// another block grew, while a copy from it was pending):
//
//   a block is never freed, regrown or rewritten while a copy from it may be pending -- the owner's
//   stream is synchronized first.
//
// HostStage tracks "may be pending" per block (`inflight`): set when a copy is enqueued from it,
// cleared when the owner's stream synchronizes (the owner calls synced() on every block it owns).
// Normal calls end with a synchronize, so the guard costs nothing on the fast path; only a call
// that left early pays one extra synchronize before the block is touched again.
//
// The owner supplies the stream and the allocator through StageOps; tests/csrc/staging_check.cpp
// drives the same code with malloc / free and a fake stream under ASan + UBSan in the CPU suite.
#ifndef KGPU_STAGING_H
#define KGPU_STAGING_H

#include <algorithm>
#include <cstddef>

namespace kgpu {

inline size_t align16(size_t bytes) { return (std::max<size_t>(bytes, 16) + 15) & ~(size_t)15; }

// Offsets of consecutive items packed into one block (each at least 16 bytes, `align`-aligned).
struct Packer {
  size_t off = 0;
  size_t place(size_t bytes, size_t align = 16) {
    const size_t o = off;
    off += (std::max<size_t>(bytes, 16) + align - 1) & ~(align - 1);
    return o;
  }
};

// What a HostStage needs from its owner.  sync() must synchronize the stream every copy from the
// owner's blocks was enqueued on and call synced() on each of those blocks.  All return 0 or a
// KGPU_E_* code.
struct StageOps {
  void* self;
  int (*sync)(void* self);
  int (*alloc)(void* self, void** p, size_t bytes);
  void (*release)(void* self, void* p);
};

struct HostStage {
  char* host = nullptr;
  size_t cap = 0;
  size_t used = 0;        // bump offset: regions handed out since the last synchronize
  bool inflight = false;  // a copy from this block may still be pending on the stream

  // A fresh region of `bytes` at the bump offset.  When the block is full it wraps -- after a
  // synchronize if a copy may be pending -- and grows (min_cap at least) when the region alone does
  // not fit; the old block is released only once nothing can read it.
  int reserve(const StageOps& ops, size_t bytes, size_t min_cap, char** out) {
    const size_t sz = align16(bytes);
    if (used + sz > cap) {
      if (inflight) {
        const int rc = ops.sync(ops.self);
        if (rc) return rc;
      }
      used = 0;
      if (sz > cap) {
        if (host) ops.release(ops.self, host);
        host = nullptr;
        cap = 0;
        const size_t want = std::max(sz * 2, min_cap);
        void* p = nullptr;
        const int rc = ops.alloc(ops.self, &p, want);
        if (rc) return rc;
        host = static_cast<char*>(p);
        cap = want;
      }
    }
    *out = host + used;
    used += sz;
    return 0;
  }

  // The block from offset 0, for an owner that rewrites the whole block every call (the query
  // pools): synchronizes first when a copy from the previous contents may be pending.
  int rewrite(const StageOps& ops, size_t bytes, size_t min_cap, char** out) {
    if (inflight) {
      const int rc = ops.sync(ops.self);
      if (rc) return rc;
    }
    used = 0;
    return reserve(ops, bytes, min_cap, out);
  }

  void enqueued() { inflight = true; }
  // the owner's stream synchronized: every copy from the block has run
  void synced() {
    inflight = false;
    used = 0;
  }
  // destruction: the owner synchronizes (or has torn the stream down) before calling this
  void release(const StageOps& ops) {
    if (host) ops.release(ops.self, host);
    host = nullptr;
    cap = used = 0;
    inflight = false;
  }
};

// The short-cycle arena: items staged in a host block at the offsets they take in a device block of
// the same layout, moved with ONE copy of the dirty range [lo, hi).  Live only inside one call
// (begin / end); begin must not run while a copy from the host block may be pending (the owner
// synchronizes when `inflight`).
struct Arena {
  bool on = false, inflight = false;
  size_t used = 0, cap = 0, lo = 0, hi = 0;

  void begin(size_t first, size_t capacity) {
    used = first;
    cap = capacity;
    on = capacity > first;
    lo = hi = 0;
  }
  void end() {
    on = false;
    lo = hi = 0;
  }
  void mark(size_t a, size_t b) {
    if (hi <= lo) {
      lo = a;
      hi = b;
    } else {
      lo = std::min(lo, a);
      hi = std::max(hi, b);
    }
  }
  // offset of a region of `bytes` (false: the arena is off or full -- the caller takes its own copy)
  bool reserve(size_t bytes, size_t* off) {
    if (!on) return false;
    const size_t o = used, sz = align16(bytes);
    if (o + sz > cap) return false;
    used = o + sz;
    mark(o, o + bytes);
    *off = o;
    return true;
  }
  // the dirty range to copy now (false: nothing); the caller enqueues it and the range resets
  bool take_dirty(size_t* a, size_t* b) {
    const bool any = hi > lo;
    *a = lo;
    *b = hi;
    lo = hi = 0;
    if (any) inflight = true;
    return any;
  }
  void synced() { inflight = false; }
};

}  // namespace kgpu

#endif  // KGPU_STAGING_H
