// ob_shard.cpp -- replicates sharded over GPUs with one RCCL all-gather of the per-replicate rows
// (replaces the Rayon `into_par_iter` of builder.rs:816-839 across devices).
//
// A replicate's row is a pure function of (seed, replicate id) and the panel (OBRS-3 counters are
// global replicate ids; the chunking depends on the panel only), so rank r simply runs replicate
// ids [first + r*per, first + (r+1)*per) on its own GPU and the gathered rows equal a one-GPU run
// bit for bit. The only collective is ncclAllGather over xGMI: (n_y x per x row_len) f64 plus
// n_y x per status bytes per rank, once per run.
//
// RCCL is bound lazily (dlopen of librccl.so.1): a process that already holds PyTorch's RCCL
// reuses that copy (same soname), and a host without RCCL still loads the engine for the
// single-GPU entry points.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "ob_common.hpp"
#include "ob_engine.hpp"
#include "ob_shard_layout.h"

static_assert(sizeof(ob_unique_id) == sizeof(ncclUniqueId), "ob_unique_id mirrors ncclUniqueId");

namespace {

#define SH_HIP(expr)                                                                                      \
  do {                                                                                                    \
    hipError_t e_ = (expr);                                                                               \
    if (e_ != hipSuccess)                                                                                 \
      return ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__);     \
  } while (0)

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;

// Resolve the RCCL entry points once; nullptr (with ob_last_error set) when RCCL is absent.
const Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!tried) {
    tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h) {
      r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
      r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
      r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
      r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
      r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
      r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
      r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
      r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
      if (r.get_unique_id && r.comm_init_rank && r.comm_init_all && r.comm_destroy && r.all_gather &&
          r.group_start && r.group_end && r.error_string)
        r.h = h;
    }
  }
  if (!r.h) {
    ob::fail(OB_E_RCCL, "RCCL (librccl.so.1) is not loadable: the multi-GPU gather needs it");
    return nullptr;
  }
  return &r;
}

int rccl_fail(const Rccl* r, ncclResult_t e, const char* what) {
  return ob::fail(OB_E_RCCL, "RCCL %s failed: %s", what, r->error_string(e));
}

#define SH_NCCL(r, expr, what)                     \
  do {                                             \
    ncclResult_t n_ = (expr);                      \
    if (n_ != ncclSuccess) return rccl_fail(r, n_, what); \
  } while (0)

void comm_free(void* c) {
  if (!c) return;
  std::lock_guard<std::mutex> lk(g_rccl_mu);  // rccl() is resolved: a communicator exists
  static ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  if (!destroy) destroy = (decltype(destroy))dlsym(RTLD_DEFAULT, "ncclCommDestroy");
  if (destroy) (void)destroy((ncclComm_t)c);
}

using Shard = ob_shard_range;

Shard shard_of(uint64_t first_rep, uint64_t n_reps, int rank, int world) {
  return ob_shard_of(first_rep, n_reps, rank, world);
}

template <typename T>
int ensure_dev(T** buf, size_t* cap, size_t elems) {
  if (*cap >= elems && *buf) return OB_OK;
  (void)hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  SH_HIP(hipMalloc(buf, sizeof(T) * std::max<size_t>(elems, 1)));
  *cap = elems;
  return OB_OK;
}

int n_gather_cols(const ob_panel* p) { return p->gather_cols.empty() ? p->row_len : (int)p->gather_cols.size(); }

// The gathered-column map on the device: [row_len] slot of each row column (-1: not gathered),
// then the nc gathered columns. Uploaded when the column set changes (a blocking copy).
int ensure_gather_map(ob_panel* p) {
  if (p->gather_map_ready) return OB_OK;
  const int rl = p->row_len, nc = n_gather_cols(p);
  std::vector<int32_t> m((size_t)rl + nc, -1);
  for (int q = 0; q < nc; ++q) {
    const int c = p->gather_cols.empty() ? q : p->gather_cols[q];
    m[c] = q;
    m[(size_t)rl + q] = c;
  }
  if (!p->d_gather_map) SH_HIP(hipMalloc(&p->d_gather_map, sizeof(int32_t) * (size_t)(2 * rl)));
  SH_HIP(hipMemcpy(p->d_gather_map, m.data(), sizeof(int32_t) * m.size(), hipMemcpyHostToDevice));
  p->gather_map_ready = true;
  return OB_OK;
}


// Enqueue this rank's shard into the panel's shard buffers, then pack the gathered columns into
// the send block and record the gather's start event.
int shard_compute(ob_panel* p, uint64_t seed, const Shard& sh, int world, int ref_mode, hipStream_t s) {
  const size_t rl = (size_t)p->row_len, ny = (size_t)p->n_y;
  const int nc = n_gather_cols(p);
  SH_HIP(hipSetDevice(p->ctx->device));
  OB_TRY(ob::engine_order(p, s));  // the previous call's gather buffers, on another stream
  OB_TRY(ensure_gather_map(p));
  const size_t slots = ny * std::max<uint64_t>(sh.per, 1);
  OB_TRY(ensure_dev(&p->d_shard_rows, &p->cap_shard, slots * rl));
  OB_TRY(ensure_dev(&p->d_shard_ok, &p->cap_shard_ok, slots));
  OB_TRY(ensure_dev(&p->d_send, &p->cap_send, slots * (size_t)nc));
  OB_TRY(ensure_dev(&p->d_send_ok, &p->cap_send_ok, slots));
  OB_TRY(ensure_dev(&p->d_gather_rows, &p->cap_gather, slots * (size_t)world * nc));
  OB_TRY(ensure_dev(&p->d_gather_ok, &p->cap_gather_ok, slots * (size_t)world));
  if (sh.count) {
    OB_TRY(ob::engine_boot(p, seed, sh.first, sh.count, ref_mode, p->d_shard_rows, p->d_shard_ok, s));
  } else if (!p->timing_pending) {  // an empty shard (n_reps < world): nothing to time but the gather
    std::memset(&p->timing, 0, sizeof(p->timing));
    p->pending_segments = 0;
    p->pending_gathers = 0;
  }
  while (p->gather_evs.size() < 2 * (size_t)(p->pending_gathers + 1)) {
    hipEvent_t e;
    SH_HIP(hipEventCreate(&e));
    p->gather_evs.push_back(e);
  }
  SH_HIP(hipEventRecord(p->gather_evs[2 * (size_t)p->pending_gathers], s));
  OB_TRY(ob::shard_pack(p->d_shard_rows, p->d_shard_ok, sh, (int)rl, nc, p->d_gather_map + rl, (int)ny, p->d_send,
                        p->d_send_ok, s));
  return OB_OK;
}

// One all-gather per outcome of the packed rows and of the ok bytes: rank r's block lands at
// ob_recv_block_off(r).
int shard_gather(const Rccl* r, ob_panel* p, ncclComm_t comm, const Shard& sh, int world, hipStream_t s) {
  const int nc = n_gather_cols(p);
  for (int t = 0; t < p->n_y; ++t) {
    SH_NCCL(r, r->all_gather(p->d_send + ob_send_off(sh, t, 0, nc, 0), p->d_gather_rows + ob_recv_block_off(sh, world, t, 0, nc),
                             ob_send_elems(sh, nc), ncclFloat64, comm, s),
            "ncclAllGather(rows)");
    SH_NCCL(r, r->all_gather(p->d_send_ok + ob_send_ok_off(sh, t, 0), p->d_gather_ok + ob_recv_block_off(sh, world, t, 0, 1),
                             sh.per, ncclUint8, comm, s),
            "ncclAllGather(ok)");
  }
  return OB_OK;
}

// Gathered blocks -> the caller's [t][n_reps] layout (device rows directly; host rows through the
// panel's staging buffers), then the gather's end event. own: this rank's shard rows (for the
// columns outside the gathered set), or the simulated rank's (ob_debug_shard_sim).
int shard_deliver(ob_panel* p, const Shard& sh, int world, uint64_t n_reps, double* rows, uint8_t* ok, bool host,
                  const double* own, hipStream_t s) {
  const size_t rl = (size_t)p->row_len, ny = (size_t)p->n_y;
  SH_HIP(hipSetDevice(p->ctx->device));
  SH_HIP(hipEventRecord(p->gather_evs[2 * (size_t)p->pending_gathers + 1], s));
  p->pending_gathers += 1;
  p->timing_pending = true;  // ob_panel_sync waits on s and reads the gather's events
  p->last_stream = s;
  double* drows = rows;
  uint8_t* dok = ok;
  if (host) {
    OB_TRY(ensure_dev(&p->d_deliver_rows, &p->cap_deliver, ny * n_reps * rl));
    OB_TRY(ensure_dev(&p->d_deliver_ok, &p->cap_deliver_ok, ny * n_reps));
    drows = p->d_deliver_rows;
    dok = p->d_deliver_ok;
  }
  OB_TRY(ob::shard_unpack(p->d_gather_rows, p->d_gather_ok, sh, world, n_reps, (int)rl, n_gather_cols(p),
                          p->d_gather_map, (int)ny, own, drows, dok, s));
  if (host) {
    SH_HIP(hipMemcpyAsync(rows, drows, sizeof(double) * ny * n_reps * rl, hipMemcpyDeviceToHost, s));
    SH_HIP(hipMemcpyAsync(ok, dok, ny * n_reps, hipMemcpyDeviceToHost, s));
  }
  return ob::engine_mark(p, s, false);  // the gather reads no count image: scratch stays as the boot left it
}

bool valid_ref(int m) { return m >= OB_REF_GROUP_A && m <= OB_REF_NEUMARK; }

int check_panel(const ob_panel* p, int ref_mode) {
  if (!valid_ref(ref_mode)) return ob::fail(OB_E_INVALID, "unknown reference coefficients %d", ref_mode);
  if (p->n[0] == 0 || p->n[1] == 0) return ob::fail(OB_E_GROUP, "%sOne group has no data", ob::error_prefix(OB_E_GROUP));
  return OB_OK;
}

int sharded_device(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode, double* d_rows,
                   uint8_t* d_ok, hipStream_t stream) {
  ob_ctx* c = p->ctx;
  hipStream_t s = stream ? stream : c->stream;
  if (!c->comm) {  // a plain context: rank 0 of 1, no collective
    OB_TRY(ob::engine_boot(p, seed, first_rep, n_reps, ref_mode, d_rows, d_ok, s));
    return OB_OK;
  }
  const Rccl* r = rccl();
  if (!r) return OB_E_RCCL;
  const Shard sh = shard_of(first_rep, n_reps, c->rank, c->world);
  OB_TRY(shard_compute(p, seed, sh, c->world, ref_mode, s));
  OB_TRY(shard_gather(r, p, (ncclComm_t)c->comm, sh, c->world, s));
  return shard_deliver(p, sh, c->world, n_reps, d_rows, d_ok, false, p->d_shard_rows, s);
}

struct Clique {
  std::vector<ncclComm_t> comms;
};
std::map<std::vector<int>, Clique> g_cliques;  // ob_boot_run_multi: one RCCL clique per device list

}  // namespace

extern "C" {

int ob_get_unique_id(ob_unique_id* id) {
  if (!id) return ob::fail(OB_E_INVALID, "null pointer");
  const Rccl* r = rccl();
  if (!r) return OB_E_RCCL;
  ncclUniqueId u;
  SH_NCCL(r, r->get_unique_id(&u), "ncclGetUniqueId");
  std::memcpy(id->internal, u.internal, sizeof(u.internal));
  return OB_OK;
}

int ob_ctx_create_rank(int device, int rank, int world, const ob_unique_id* id, ob_ctx** out) {
  if (!id || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return ob::fail(OB_E_INVALID, "rank %d of world %d", rank, world);
  const Rccl* r = rccl();
  if (!r) return OB_E_RCCL;
  ob_ctx* c = nullptr;
  OB_TRY(ob_ctx_create(device, &c));
  ncclUniqueId u;
  std::memcpy(u.internal, id->internal, sizeof(u.internal));
  ncclComm_t comm = nullptr;
  SH_HIP(hipSetDevice(device));
  const ncclResult_t e = r->comm_init_rank(&comm, world, u, rank);
  if (e != ncclSuccess) {
    ob_ctx_destroy(c);
    return rccl_fail(r, e, "ncclCommInitRank");
  }
  c->rank = rank;
  c->world = world;
  c->comm = comm;
  c->comm_free = comm_free;
  *out = c;
  return OB_OK;
}

int ob_ctx_rank(const ob_ctx* c, int* rank, int* world) {
  if (!c || !rank || !world) return ob::fail(OB_E_INVALID, "null pointer");
  *rank = c->rank;
  *world = c->world;
  return OB_OK;
}

int ob_boot_run_sharded_device(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                               double* d_rows, uint8_t* d_ok, void* hip_stream) {
  if (!p || (n_reps && (!d_rows || !d_ok))) return ob::fail(OB_E_INVALID, "null pointer");
  OB_TRY(check_panel(p, ref_mode));
  if (n_reps == 0) return OB_OK;
  return sharded_device(p, seed, first_rep, n_reps, ref_mode, d_rows, d_ok, reinterpret_cast<hipStream_t>(hip_stream));
}

int ob_boot_run_sharded(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode, double* rows,
                        uint8_t* ok) {
  if (!p || (n_reps && (!rows || !ok))) return ob::fail(OB_E_INVALID, "null pointer");
  OB_TRY(check_panel(p, ref_mode));
  if (n_reps == 0) return OB_OK;
  ob_ctx* c = p->ctx;
  if (!c->comm) return ob_boot_run(p, seed, first_rep, n_reps, ref_mode, rows, ok);
  const Rccl* r = rccl();
  if (!r) return OB_E_RCCL;
  const Shard sh = shard_of(first_rep, n_reps, c->rank, c->world);
  OB_TRY(shard_compute(p, seed, sh, c->world, ref_mode, c->stream));
  OB_TRY(shard_gather(r, p, (ncclComm_t)c->comm, sh, c->world, c->stream));
  OB_TRY(shard_deliver(p, sh, c->world, n_reps, rows, ok, true, p->d_shard_rows, c->stream));
  return ob_panel_sync(p);
}

int ob_boot_run_multi(ob_panel* const* panels, int n_panels, uint64_t seed, uint64_t first_rep, uint64_t n_reps,
                      int ref_mode, double* rows, uint8_t* ok) {
  if (!panels || n_panels < 1 || (n_reps && (!rows || !ok))) return ob::fail(OB_E_INVALID, "bad arguments");
  std::vector<int> devs(n_panels);
  for (int i = 0; i < n_panels; ++i) {
    if (!panels[i]) return ob::fail(OB_E_INVALID, "null panel %d", i);
    OB_TRY(check_panel(panels[i], ref_mode));
    const ob_panel* p0 = panels[0];
    const ob_panel* pi = panels[i];
    if (pi->row_len != p0->row_len || pi->n_y != p0->n_y || pi->n[0] != p0->n[0] || pi->n[1] != p0->n[1] ||
        pi->p != p0->p)
      return ob::fail(OB_E_INVALID, "panel %d does not hold the same design as panel 0", i);
    if (pi->gather_cols != p0->gather_cols)
      return ob::fail(OB_E_INVALID, "panel %d gathers other columns than panel 0", i);
    devs[i] = pi->ctx->device;
    for (int j = 0; j < i; ++j)
      if (devs[j] == devs[i]) return ob::fail(OB_E_INVALID, "panels %d and %d share device %d", j, i, devs[i]);
  }
  if (n_reps == 0) return OB_OK;
  const Rccl* r = rccl();
  if (!r) return OB_E_RCCL;
  Clique* cq = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    auto it = g_cliques.find(devs);
    if (it == g_cliques.end()) {
      Clique c;
      c.comms.resize(n_panels);
      const ncclResult_t e = r->comm_init_all(c.comms.data(), n_panels, devs.data());
      if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommInitAll");
      it = g_cliques.emplace(devs, std::move(c)).first;
    }
    cq = &it->second;
  }
  std::vector<Shard> sh(n_panels);
  for (int i = 0; i < n_panels; ++i) {
    sh[i] = shard_of(first_rep, n_reps, i, n_panels);
    OB_TRY(shard_compute(panels[i], seed, sh[i], n_panels, ref_mode, panels[i]->ctx->stream));
  }
  SH_NCCL(r, r->group_start(), "ncclGroupStart");
  int rc = OB_OK;
  for (int i = 0; i < n_panels && rc == OB_OK; ++i)
    rc = shard_gather(r, panels[i], cq->comms[i], sh[i], n_panels, panels[i]->ctx->stream);
  SH_NCCL(r, r->group_end(), "ncclGroupEnd");
  OB_TRY(rc);
  ob_panel* p0 = panels[0];
  OB_TRY(shard_deliver(p0, sh[0], n_panels, n_reps, rows, ok, true, p0->d_shard_rows, p0->ctx->stream));
  for (int i = 0; i < n_panels; ++i) OB_TRY(ob_panel_sync(panels[i]));
  return OB_OK;
}

int ob_panel_set_gather_columns(ob_panel* p, const int32_t* cols, int32_t n) {
  if (!p || (n > 0 && !cols) || n < 0) return ob::fail(OB_E_INVALID, "bad arguments");
  std::vector<int32_t> v(cols, cols + n);
  for (int32_t i = 0; i < n; ++i)
    if (v[i] < 0 || v[i] >= p->row_len || (i && v[i] <= v[i - 1]))
      return ob::fail(OB_E_INVALID, "gather columns must be ascending row offsets in [0, %d)", p->row_len);
  if ((int)v.size() == p->row_len) v.clear();  // every column
  if (v != p->gather_cols) {
    p->gather_cols = std::move(v);
    p->gather_map_ready = false;
  }
  return OB_OK;
}

int ob_debug_shard_sim(ob_panel* p, int world, int self_rank, uint64_t seed, uint64_t first_rep, uint64_t n_reps,
                       int ref_mode, double* rows, uint8_t* ok) {
  if (!p || world < 1 || self_rank < 0 || self_rank >= world || (n_reps && (!rows || !ok)))
    return ob::fail(OB_E_INVALID, "bad arguments");
  OB_TRY(check_panel(p, ref_mode));
  if (n_reps == 0) return OB_OK;
  hipStream_t s = p->ctx->stream;
  const size_t rl = (size_t)p->row_len, ny = (size_t)p->n_y;
  const int nc = n_gather_cols(p);
  Shard self{};
  for (int r = 0; r < world; ++r) {
    const Shard sh = shard_of(first_rep, n_reps, r, world);
    OB_TRY(shard_compute(p, seed, sh, world, ref_mode, s));
    OB_TRY(ob::engine_collect(p));  // this rank's shard has finished (its ok / overflow checks)
    for (int t = 0; t < p->n_y; ++t) {  // the all-gather's placement of rank r's blocks
      SH_HIP(hipMemcpyAsync(p->d_gather_rows + ob_recv_block_off(sh, world, t, r, nc), p->d_send + ob_send_off(sh, t, 0, nc, 0),
                            sizeof(double) * ob_send_elems(sh, nc), hipMemcpyDeviceToDevice, s));
      SH_HIP(hipMemcpyAsync(p->d_gather_ok + ob_recv_block_off(sh, world, t, r, 1), p->d_send_ok + ob_send_ok_off(sh, t, 0),
                            sh.per, hipMemcpyDeviceToDevice, s));
    }
    if (r == self_rank) {
      self = sh;
      OB_TRY(ensure_dev(&p->d_own_rows, &p->cap_own, std::max<size_t>(ny * sh.count * rl, 1)));
      if (sh.count)
        SH_HIP(hipMemcpyAsync(p->d_own_rows, p->d_shard_rows, sizeof(double) * ny * sh.count * rl, hipMemcpyDeviceToDevice, s));
    }
  }
  OB_TRY(shard_deliver(p, self, world, n_reps, rows, ok, true, p->d_own_rows, s));
  return ob_panel_sync(p);
}

}  // extern "C"

namespace ob {

void shard_free(ob_panel* p) {
  (void)hipFree(p->d_shard_rows);
  (void)hipFree(p->d_shard_ok);
  (void)hipFree(p->d_send);
  (void)hipFree(p->d_send_ok);
  (void)hipFree(p->d_gather_rows);
  (void)hipFree(p->d_gather_ok);
  (void)hipFree(p->d_deliver_rows);
  (void)hipFree(p->d_deliver_ok);
  (void)hipFree(p->d_own_rows);
  (void)hipFree(p->d_gather_map);
  for (hipEvent_t e : p->gather_evs) (void)hipEventDestroy(e);
  p->gather_evs.clear();
}

}  // namespace ob
