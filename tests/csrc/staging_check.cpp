// Host-staging bookkeeping of libkgpu (kubernetes-1_amd/csrc/kgpu_staging.h) under ASan + UBSan,
// driven by a fake stream: a copy enqueued from a staging block runs only at the next synchronize,
// reading the block THEN, as hipMemcpyAsync from pinned memory does.  Each copy also snapshots the
// bytes at enqueue time, so a block rewritten before its copy ran is caught even when the memory is
// still allocated; a block freed before its copy ran is a heap-use-after-free for ASan.
//
//   staging_check            every scenario, "staging ok" on success
//   staging_check unsafe     the round-3 bug on purpose (a block freed while a copy from it is
//                            pending): must die under ASan -- proves the harness catches it
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "kgpu_staging.h"

namespace {

struct Copy {
  const char* src;
  size_t n;
  std::vector<char> expect;
};

struct Owner {
  std::vector<Copy> pending;
  std::vector<kgpu::HostStage*> stages;
  kgpu::Arena* arena = nullptr;
  std::vector<char> device = std::vector<char>(8 << 20);
  long syncs = 0, allocs = 0, frees = 0;

  void enqueue(const char* src, size_t n) { pending.push_back(Copy{src, n, std::vector<char>(src, src + n)}); }
  void run() {
    for (const Copy& c : pending) {
      std::memcpy(device.data(), c.src, std::min(c.n, device.size()));  // reads the block now
      if (std::memcmp(c.src, c.expect.data(), c.n) != 0) {
        std::fprintf(stderr, "FAIL: a staging block was rewritten before its pending copy ran\n");
        std::abort();
      }
    }
    pending.clear();
  }
};

int o_sync(void* self) {
  Owner* o = static_cast<Owner*>(self);
  o->run();
  for (kgpu::HostStage* s : o->stages) s->synced();
  if (o->arena) o->arena->synced();
  ++o->syncs;
  return 0;
}
int o_alloc(void* self, void** p, size_t n) {
  ++static_cast<Owner*>(self)->allocs;
  *p = std::malloc(n);
  return *p ? 0 : -2;
}
void o_release(void* self, void* p) {
  ++static_cast<Owner*>(self)->frees;
  std::free(p);
}

void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    std::exit(1);
  }
}

void fill(char* p, size_t n, unsigned tag) {
  for (size_t i = 0; i < n; ++i) p[i] = static_cast<char>((tag * 131u + i) & 0xFF);
}

// round 3: the query-pool block was freed while a copy from it was pending (another block grew);
// here the pool block itself regrows with its previous copy still pending
void regrow_with_pending_copy() {
  Owner o;
  kgpu::HostStage pool, tables;
  o.stages = {&pool, &tables};
  const kgpu::StageOps ops{&o, o_sync, o_alloc, o_release};
  char* h = nullptr;
  check(pool.rewrite(ops, 200, 256, &h) == 0, "pool rewrite");
  fill(h, 200, 1);
  o.enqueue(h, 200);
  pool.enqueued();
  // the table block grows while the pool copy is pending: the pool block must stay untouched
  check(tables.reserve(ops, 4096, 1024, &h) == 0, "tables reserve");
  fill(h, 4096, 2);
  o.enqueue(h, 4096);
  tables.enqueued();
  // a call that left early (no synchronize), then a bigger pool: regrow -> synchronize first
  check(pool.rewrite(ops, 1 << 20, 256, &h) == 0, "pool regrow");
  check(o.pending.empty(), "the regrow synchronized before freeing the old block");
  fill(h, 1 << 20, 3);
  o.enqueue(h, 1 << 20);
  pool.enqueued();
  o_sync(&o);
  pool.release(ops);
  tables.release(ops);
  check(o.allocs == o.frees, "every staging block released once");
}

// upload_pools rewrote its block without synchronizing after an error exit
void rewrite_after_error_exit() {
  Owner o;
  kgpu::HostStage pool;
  o.stages = {&pool};
  const kgpu::StageOps ops{&o, o_sync, o_alloc, o_release};
  char* h = nullptr;
  check(pool.rewrite(ops, 512, 4096, &h) == 0, "rewrite 1");
  fill(h, 512, 4);
  o.enqueue(h, 512);
  pool.enqueued();
  // the call fails before its synchronize; the next call rewrites the same bytes
  const long s0 = o.syncs;
  check(pool.rewrite(ops, 512, 4096, &h) == 0, "rewrite 2");
  check(o.syncs == s0 + 1, "a rewrite with a pending copy synchronizes first");
  fill(h, 512, 5);
  // the normal path pays nothing: no pending copy, no synchronize
  o_sync(&o);
  const long s1 = o.syncs;
  check(pool.rewrite(ops, 512, 4096, &h) == 0, "rewrite 3");
  check(o.syncs == s1, "no synchronize without a pending copy");
  pool.release(ops);
}

// bump allocation wraps only after a synchronize
void bump_wraps_after_sync() {
  Owner o;
  kgpu::HostStage t;
  o.stages = {&t};
  const kgpu::StageOps ops{&o, o_sync, o_alloc, o_release};
  char* h = nullptr;
  check(t.reserve(ops, 1000, 4096, &h) == 0, "first");  // cap 4096
  for (unsigned k = 0; k < 40; ++k) {
    check(t.reserve(ops, 1000, 4096, &h) == 0, "reserve");
    check(h >= t.host && h + 1000 <= t.host + t.cap, "region inside the block");
    fill(h, 1000, 10 + k);
    o.enqueue(h, 1000);
    t.enqueued();
  }
  o_sync(&o);
  t.release(ops);
}

void arena_ranges() {
  kgpu::Arena a;
  a.begin(1024, 1024 + 4096);
  size_t off[8];
  for (int i = 0; i < 8; ++i) check(a.reserve(100 + 37 * i, &off[i]), "arena reserve");
  for (int i = 1; i < 8; ++i) check(off[i] >= off[i - 1] + 100 + 37 * (i - 1), "arena items do not overlap");
  size_t lo, hi;
  check(a.take_dirty(&lo, &hi) && lo == off[0] && hi == off[7] + 100 + 37 * 7, "dirty range covers every item");
  check(a.inflight && !a.take_dirty(&lo, &hi), "the range resets after the copy is taken");
  size_t big;
  check(!a.reserve(8192, &big), "an item larger than the arena takes its own copy");
  a.end();
  check(!a.reserve(16, &big), "no arena outside a call");
  kgpu::Arena off0;
  off0.begin(1024, 0);
  check(!off0.on, "KGPU_OPT_ARENA_BYTES = 0 turns the arena off");
  kgpu::Packer p;
  const size_t a0 = p.place(3), a1 = p.place(40), a2 = p.place(0), a3 = p.place(100, 64);
  check(a0 == 0 && a1 == 16 && a2 == 64 && a3 == 80 && p.off == 80 + 128, "packed offsets");
}

// seeded interleavings of the three blocks the library owns (pools rewrite, tables and deltas bump /
// rewrite), random sizes across the growth thresholds, random early exits (no synchronize)
void fuzz(unsigned seed) {
  std::mt19937 r(seed);
  Owner o;
  kgpu::HostStage pool, tables, delta;
  kgpu::Arena ar;
  o.stages = {&pool, &tables, &delta};
  o.arena = &ar;
  const kgpu::StageOps ops{&o, o_sync, o_alloc, o_release};
  for (int it = 0; it < 4000; ++it) {
    const size_t n = 1 + r() % (r() % 8 == 0 ? (1u << 18) : 3000u);
    char* h = nullptr;
    const unsigned which = r() % 3;
    kgpu::HostStage& s = which == 0 ? pool : which == 1 ? tables : delta;
    const int rc = which == 1 ? s.reserve(ops, n, 1 << 12, &h) : s.rewrite(ops, n, 1 << 12, &h);
    check(rc == 0, "stage");
    check(h >= s.host && h + n <= s.host + s.cap, "region inside its block");
    fill(h, n, (unsigned)it);
    if (r() % 4) {
      o.enqueue(h, n);
      s.enqueued();
    }
    if (r() % 5 == 0) o_sync(&o);  // a call that ran to its end
  }
  o_sync(&o);
  pool.release(ops);
  tables.release(ops);
  delta.release(ops);
  check(o.allocs == o.frees, "fuzz: every block released once");
}

// the harness must catch the round-3 bug: free a block with a copy from it still pending
void unsafe() {
  Owner o;
  char* h = static_cast<char*>(std::malloc(256));
  fill(h, 256, 9);
  o.enqueue(h, 256);
  std::free(h);  // what a regrow without the synchronize did
  o.run();       // the copy reads freed memory: ASan aborts here
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "unsafe") == 0) {
    unsafe();
    std::printf("unsafe run finished without a report\n");
    return 0;
  }
  regrow_with_pending_copy();
  rewrite_after_error_exit();
  bump_wraps_after_sync();
  arena_ranges();
  for (unsigned seed = 1; seed <= 8; ++seed) fuzz(seed);
  std::printf("staging ok\n");
  return 0;
}
