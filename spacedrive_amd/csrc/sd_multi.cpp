// sd_multi.cpp — single-process multi-device Object grouping and end-to-end hashing
// (C ABI sd_cas_multi_*).
//
// The Rust core is one process; it drives every local MI355X itself.  Files shard by
// contiguous index range, one shard per device context (a device may host several shards,
// which is how the exchange is tested on a one-GPU box).  Grouping:
//   1. per shard: stable radix sort of (key, local idx); split points of the key ranges
//      dest(k) = floor(k * G / 2^64) by binary search on the sorted keys;
//   2. exchange: every shard PULLS its key range from every other shard with
//      hipMemcpyPeerAsync over xGMI on its own stream, ordered after the sources' sorts by
//      cross-device events (no collective library needed inside one process; the
//      multi-process path uses RCCL, spacedrive_amd/shard.py);
//   3. per shard: sort the received (key, position), group runs; the head of a run is the
//      global minimum file idx because runs arrive in shard order and each run is
//      idx-ascending (file0 must ascend across shards);
//   4. mirror pull of the representatives, scatter into local order.
#include <hip/hip_runtime.h>
#include <string.h>

#include <vector>

#include "ctx_internal.h"
#include "sd_group.h"
#include "sd_kernels.h"
#include "sd_multi.h"

using namespace sdcas;

struct sd_cas_multi {
  int G = 0;
  std::vector<sd_cas_ctx*> ctx;
  std::vector<hipEvent_t> ev_a, ev_b;
  uint64_t* h_splits = nullptr;  // pinned [G][G+1]
  std::string err;
};

static int mfail(sd_cas_multi* m, int code, const std::string& what) {
  if (m) m->err = what;
  return code;
}

// why the last sd_cas_multi_create on this thread failed (sd_cas_multi_last_error(NULL))
static thread_local std::string g_create_err;

#define MTRY(m, i, expr)                                                                   \
  do {                                                                                     \
    int rc_ = (expr);                                                                      \
    if (rc_ != SD_CAS_OK)                                                                  \
      return mfail((m), rc_, std::string("shard ") + std::to_string(i) + ": " +           \
                                 sd_cas_last_error((m)->ctx[i]));                          \
  } while (0)

#define MHIP(m, i, expr)                                                                   \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return mfail((m), SD_CAS_EHIP, std::string("shard ") + std::to_string(i) + ": " + #expr + \
                                         ": " + hipGetErrorString(e_));                     \
  } while (0)

// per-shard exchange buffers in ctx->small
struct Bufs {
  uint64_t* skeys; uint32_t* sidx; uint64_t* gidx; uint64_t* splits; uint64_t* back;
  uint64_t* rkeys; uint64_t* ridx; uint64_t* k2; uint32_t* pos; uint32_t* rep_pos; uint64_t* repg;
};

static size_t bufs_bytes(size_t n, size_t m, int G) {
  return up256(n * 8) + up256(n * 4) + up256(n * 8) + up256((G + 1) * 8) + up256(n * 8) +
         up256(m * 8) * 2 + up256(m * 8) + up256(m * 4) * 2 + up256(m * 8) + 256;
}

static Bufs carve(void* base, size_t n, size_t m, int G) {
  char* p = (char*)base;
  Bufs b;
  b.skeys = (uint64_t*)p; p += up256(n * 8);
  b.sidx = (uint32_t*)p; p += up256(n * 4);
  b.gidx = (uint64_t*)p; p += up256(n * 8);
  b.splits = (uint64_t*)p; p += up256((G + 1) * 8);
  b.back = (uint64_t*)p; p += up256(n * 8);
  b.rkeys = (uint64_t*)p; p += up256(m * 8);
  b.ridx = (uint64_t*)p; p += up256(m * 8);
  b.k2 = (uint64_t*)p; p += up256(m * 8);
  b.pos = (uint32_t*)p; p += up256(m * 4);
  b.rep_pos = (uint32_t*)p; p += up256(m * 4);
  b.repg = (uint64_t*)p;
  return b;
}

extern "C" {

int sd_cas_multi_create(const int* devices, int ndev, sd_cas_multi** out) {
  if (!devices || ndev <= 0 || ndev > 64 || !out) return SD_CAS_EINVAL;
  *out = nullptr;
  g_create_err.clear();
  sd_cas_multi* m = new sd_cas_multi();
  m->G = ndev;
  for (int i = 0; i < ndev; i++) {
    sd_cas_ctx* c = nullptr;
    int rc = sd_cas_ctx_create(devices[i], &c);
    if (rc) {
      g_create_err = "shard " + std::to_string(i) + ": no gfx950 device " + std::to_string(devices[i]);
      sd_cas_multi_destroy(m);
      return rc;
    }
    m->ctx.push_back(c);
  }
  // peer access between distinct devices (the exchange pulls over xGMI); a shard pair on
  // one device copies D2D.  Without peer access the pulls would silently stage through
  // host memory, so a pair that cannot be enabled fails the creation.
  for (int i = 0; i < ndev; i++)
    for (int j = 0; j < ndev; j++) {
      if (devices[i] == devices[j]) continue;
      int can = 0;
      hipError_t e = hipDeviceCanAccessPeer(&can, devices[i], devices[j]);
      if (e == hipSuccess && can) {
        e = hipSetDevice(devices[i]);
        if (e == hipSuccess) e = hipDeviceEnablePeerAccess(devices[j], 0);
        if (e == hipErrorPeerAccessAlreadyEnabled) e = hipSuccess;
      }
      (void)hipGetLastError();
      if (e != hipSuccess || !can) {
        g_create_err = "peer access " + std::to_string(devices[i]) + " -> " + std::to_string(devices[j]) +
                       (e != hipSuccess ? std::string(": ") + hipGetErrorString(e) : ": not supported");
        sd_cas_multi_destroy(m);
        return SD_CAS_ENODEV;
      }
    }
  m->ev_a.resize(ndev);
  m->ev_b.resize(ndev);
  for (int i = 0; i < ndev; i++) {
    (void)hipSetDevice(devices[i]);
    if (hipEventCreateWithFlags(&m->ev_a[i], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_b[i], hipEventDisableTiming) != hipSuccess) {
      sd_cas_multi_destroy(m);
      return SD_CAS_EHIP;
    }
  }
  if (hipHostMalloc((void**)&m->h_splits, (size_t)ndev * (ndev + 1) * 8, hipHostMallocDefault) !=
      hipSuccess) {
    sd_cas_multi_destroy(m);
    return SD_CAS_ENOMEM;
  }
  *out = m;
  return SD_CAS_OK;
}

void sd_cas_multi_destroy(sd_cas_multi* m) {
  if (!m) return;
  for (size_t i = 0; i < m->ctx.size(); i++) {
    (void)hipSetDevice(m->ctx[i]->device);
    if (i < m->ev_a.size() && m->ev_a[i]) (void)hipEventDestroy(m->ev_a[i]);
    if (i < m->ev_b.size() && m->ev_b[i]) (void)hipEventDestroy(m->ev_b[i]);
  }
  for (auto* c : m->ctx) sd_cas_ctx_destroy(c);
  if (m->h_splits) (void)hipHostFree(m->h_splits);
  delete m;
}

int sd_cas_multi_count(const sd_cas_multi* m) { return m ? m->G : 0; }

sd_cas_ctx* sd_cas_multi_ctx(sd_cas_multi* m, int i) {
  return (m && i >= 0 && i < m->G) ? m->ctx[i] : nullptr;
}

const char* sd_cas_multi_last_error(const sd_cas_multi* m) {
  return m ? m->err.c_str() : g_create_err.c_str();
}

int sd_cas_multi_group(sd_cas_multi* m, const uint64_t* const* d_keys, const size_t* n,
                       const uint64_t* file0, uint64_t* const* d_rep, uint64_t* out_objects) {
  if (!m || !d_keys || !n || !file0 || !d_rep) return SD_CAS_EINVAL;
  const int G = m->G;
  for (int i = 0; i < G; i++) {
    if (n[i] >= (1ull << 32) || (n[i] && (!d_keys[i] || !d_rep[i])))
      return mfail(m, SD_CAS_EINVAL, "bad shard arguments");
    if (i && file0[i] < file0[i - 1] + n[i - 1])
      return mfail(m, SD_CAS_EINVAL, "file0 must ascend with disjoint shard ranges");
  }
  // 1. local sorts + split points (counts come back to the host: one sync)
  std::vector<size_t> cap(G);
  for (int i = 0; i < G; i++) {
    sd_cas_ctx* c = m->ctx[i];
    MHIP(m, i, hipSetDevice(c->device));
    // receive side unknown yet: size for n_i now, regrow after the counts are known
    MTRY(m, i, sd_ensure(c, c->small, bufs_bytes(n[i], n[i], G)));
    Bufs b = carve(c->small.p, n[i], n[i], G);
    if (n[i]) MTRY(m, i, sd_cas_sort_pairs_dev(c, d_keys[i], nullptr, n[i], b.skeys, b.sidx, 0, 64, c->stream));
    MHIP(m, i, multi_splits(b.skeys, n[i], (uint32_t)G, b.splits, c->stream));
    MHIP(m, i, multi_gidx(b.sidx, n[i], file0[i], b.gidx, c->stream));
    MHIP(m, i, hipMemcpyAsync(m->h_splits + (size_t)i * (G + 1), b.splits, (G + 1) * 8,
                              hipMemcpyDeviceToHost, c->stream));
  }
  for (int i = 0; i < G; i++) {
    MHIP(m, i, hipSetDevice(m->ctx[i]->device));
    MHIP(m, i, hipStreamSynchronize(m->ctx[i]->stream));
  }
  auto cnt = [&](int i, int j) { return m->h_splits[(size_t)i * (G + 1) + j + 1] - m->h_splits[(size_t)i * (G + 1) + j]; };
  auto off = [&](int i, int j) { return m->h_splits[(size_t)i * (G + 1) + j]; };
  std::vector<size_t> recv(G, 0);
  std::vector<std::vector<size_t>> roff(G, std::vector<size_t>(G, 0));
  for (int j = 0; j < G; j++)
    for (int i = 0; i < G; i++) { roff[j][i] = recv[j]; recv[j] += cnt(i, j); }
  // grow the exchange buffers to the received sizes (keeps the sorted data: copy it over)
  for (int i = 0; i < G; i++) {
    sd_cas_ctx* c = m->ctx[i];
    const size_t need = bufs_bytes(n[i], recv[i], G);
    if (need > c->small.bytes) {
      MHIP(m, i, hipSetDevice(c->device));
      DevBuf nb;
      MTRY(m, i, sd_ensure(c, nb, need));
      Bufs ob = carve(c->small.p, n[i], n[i], G), nw = carve(nb.p, n[i], recv[i], G);
      MHIP(m, i, hipMemcpyAsync(nw.skeys, ob.skeys, n[i] * 8, hipMemcpyDeviceToDevice, c->stream));
      MHIP(m, i, hipMemcpyAsync(nw.sidx, ob.sidx, n[i] * 4, hipMemcpyDeviceToDevice, c->stream));
      MHIP(m, i, hipMemcpyAsync(nw.gidx, ob.gidx, n[i] * 8, hipMemcpyDeviceToDevice, c->stream));
      MHIP(m, i, hipStreamSynchronize(c->stream));
      MHIP(m, i, hipFree(c->small.p));
      c->small = nb;
    }
  }
  std::vector<Bufs> B(G);
  for (int i = 0; i < G; i++) {
    B[i] = carve(m->ctx[i]->small.p, n[i], recv[i], G);
    MHIP(m, i, hipSetDevice(m->ctx[i]->device));
    MHIP(m, i, hipEventRecord(m->ev_a[i], m->ctx[i]->stream));
  }
  // 2. exchange (pull) + 3. local grouping of the received key range
  std::vector<uint64_t> objects(G, 0);
  for (int j = 0; j < G; j++) {
    sd_cas_ctx* c = m->ctx[j];
    MHIP(m, j, hipSetDevice(c->device));
    for (int i = 0; i < G; i++) {
      const size_t k = cnt(i, j);
      if (!k) continue;
      MHIP(m, j, hipStreamWaitEvent(c->stream, m->ev_a[i], 0));
      MHIP(m, j, hipMemcpyPeerAsync(B[j].rkeys + roff[j][i], c->device, B[i].skeys + off(i, j),
                                    m->ctx[i]->device, k * 8, c->stream));
      MHIP(m, j, hipMemcpyPeerAsync(B[j].ridx + roff[j][i], c->device, B[i].gidx + off(i, j),
                                    m->ctx[i]->device, k * 8, c->stream));
    }
    if (recv[j]) {
      MTRY(m, j, sd_cas_sort_pairs_dev(c, B[j].rkeys, nullptr, recv[j], B[j].k2, B[j].pos, 0, 64, c->stream));
      MTRY(m, j, sd_cas_group_sorted_dev(c, B[j].k2, B[j].pos, recv[j], B[j].rep_pos, nullptr, c->stream));
      MHIP(m, j, hipMemcpyAsync(c->d_scalar + 7, c->d_scalar, 8, hipMemcpyDeviceToDevice, c->stream));
      MHIP(m, j, multi_gather(B[j].rep_pos, B[j].ridx, recv[j], B[j].repg, c->stream));
    }
    MHIP(m, j, hipEventRecord(m->ev_b[j], c->stream));
  }
  // 4. mirror pull of the representatives, scatter into local order
  for (int i = 0; i < G; i++) {
    sd_cas_ctx* c = m->ctx[i];
    MHIP(m, i, hipSetDevice(c->device));
    for (int j = 0; j < G; j++) {
      const size_t k = cnt(i, j);
      if (!k) continue;
      MHIP(m, i, hipStreamWaitEvent(c->stream, m->ev_b[j], 0));
      MHIP(m, i, hipMemcpyPeerAsync(B[i].back + off(i, j), c->device, B[j].repg + roff[j][i],
                                    m->ctx[j]->device, k * 8, c->stream));
    }
    MHIP(m, i, multi_scatter(B[i].sidx, B[i].back, n[i], d_rep[i], c->stream));
  }
  uint64_t total = 0;
  for (int i = 0; i < G; i++) {
    sd_cas_ctx* c = m->ctx[i];
    MHIP(m, i, hipSetDevice(c->device));
    if (recv[i]) {
      MHIP(m, i, hipMemcpyAsync(&objects[i], c->d_scalar + 7, 8, hipMemcpyDeviceToHost, c->stream));
    }
    MHIP(m, i, hipStreamSynchronize(c->stream));
    total += objects[i];
  }
  if (out_objects) *out_objects = total;
  return SD_CAS_OK;
}

int sd_cas_multi_hash_group_sampled_host(sd_cas_multi* m, const void* h_content, uint64_t stride,
                                         const uint64_t* h_sizes, size_t n, uint64_t* h_keys,
                                         uint64_t* h_rep, uint64_t* out_objects) {
  if (!m || (n && (!h_content || !h_sizes || !h_keys))) return SD_CAS_EINVAL;
  if (stride < SD_CAS_SAMPLED_CONTENT_LEN || (stride & 15))
    return mfail(m, SD_CAS_EINVAL, "bad stride");
  const int G = m->G;
  std::vector<size_t> ns(G), f0(G);
  std::vector<DevBuf> keys(G), rep(G);
  for (int i = 0; i < G; i++) {
    f0[i] = n * (size_t)i / G;
    ns[i] = n * (size_t)(i + 1) / G - f0[i];
  }
  // hash every shard from host memory: batches ping-pong between H2D on the side stream
  // and K1 on the compute stream, all devices in flight together
  const size_t batch = sd_cas_batch_quantum(m->ctx[0]);
  const size_t cbytes = up256(batch * stride), sbytes = up256(batch * 8);
  for (int i = 0; i < G; i++) {
    sd_cas_ctx* c = m->ctx[i];
    MHIP(m, i, hipSetDevice(c->device));
    MTRY(m, i, sd_ensure(c, c->staging, 2 * (cbytes + sbytes)));
    MTRY(m, i, sd_ensure(c, keys[i], ns[i] * 8 + 256));
    MTRY(m, i, sd_ensure(c, rep[i], ns[i] * 8 + 256));
  }
  std::vector<hipEvent_t> h2d(2 * G), done(2 * G);
  for (int i = 0; i < G; i++) {
    MHIP(m, i, hipSetDevice(m->ctx[i]->device));
    for (int s = 0; s < 2; s++) {
      MHIP(m, i, hipEventCreateWithFlags(&h2d[2 * i + s], hipEventDisableTiming));
      MHIP(m, i, hipEventCreateWithFlags(&done[2 * i + s], hipEventDisableTiming));
    }
  }
  size_t maxb = 0;
  for (int i = 0; i < G; i++) maxb = std::max(maxb, (ns[i] + batch - 1) / batch);
  int result = SD_CAS_OK;
  for (size_t k = 0; k < maxb && result == SD_CAS_OK; k++) {
    for (int i = 0; i < G; i++) {
      if (k * batch >= ns[i]) continue;
      sd_cas_ctx* c = m->ctx[i];
      const int s = (int)(k & 1);
      const size_t b0 = f0[i] + k * batch, cntf = std::min(batch, ns[i] - k * batch);
      char* slot = (char*)c->staging.p + s * (cbytes + sbytes);
      hipError_t e = hipSetDevice(c->device);
      if (e == hipSuccess && k >= 2) e = hipStreamWaitEvent(c->copy, done[2 * i + s], 0);
      if (e == hipSuccess)
        e = hipMemcpyAsync(slot, (const char*)h_content + b0 * stride, cntf * stride,
                           hipMemcpyHostToDevice, c->copy);
      if (e == hipSuccess)
        e = hipMemcpyAsync(slot + cbytes, h_sizes + b0, cntf * 8, hipMemcpyHostToDevice, c->copy);
      if (e == hipSuccess) e = hipEventRecord(h2d[2 * i + s], c->copy);
      if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, h2d[2 * i + s], 0);
      if (e == hipSuccess)
        e = hash_sampled((const uint8_t*)slot, stride, (const uint64_t*)(slot + cbytes), cntf,
                         (uint64_t*)keys[i].p + k * batch, c->stream,
                         (uint32_t)(sd_cas_batch_quantum(c) / 256));
      if (e == hipSuccess) e = hipEventRecord(done[2 * i + s], c->stream);
      if (e != hipSuccess)
        result = mfail(m, SD_CAS_EHIP, std::string("hash shard ") + std::to_string(i) + ": " +
                                           hipGetErrorString(e));
    }
  }
  if (result == SD_CAS_OK) {
    std::vector<const uint64_t*> dk(G);
    std::vector<uint64_t*> dr(G);
    std::vector<uint64_t> file0(G);
    for (int i = 0; i < G; i++) { dk[i] = (const uint64_t*)keys[i].p; dr[i] = (uint64_t*)rep[i].p; file0[i] = f0[i]; }
    result = sd_cas_multi_group(m, dk.data(), ns.data(), file0.data(), dr.data(), out_objects);
  }
  for (int i = 0; i < G && result == SD_CAS_OK; i++) {
    sd_cas_ctx* c = m->ctx[i];
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess && ns[i])
      e = hipMemcpyAsync(h_keys + f0[i], keys[i].p, ns[i] * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && ns[i] && h_rep)
      e = hipMemcpyAsync(h_rep + f0[i], rep[i].p, ns[i] * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) result = mfail(m, SD_CAS_EHIP, hipGetErrorString(e));
  }
  for (int i = 0; i < G; i++) {
    (void)hipSetDevice(m->ctx[i]->device);
    (void)hipStreamSynchronize(m->ctx[i]->stream);
    (void)hipStreamSynchronize(m->ctx[i]->copy);
    for (int s = 0; s < 2; s++) {
      (void)hipEventDestroy(h2d[2 * i + s]);
      (void)hipEventDestroy(done[2 * i + s]);
    }
    if (keys[i].p) (void)hipFree(keys[i].p);
    if (rep[i].p) (void)hipFree(rep[i].p);
  }
  return result;
}

// ---- row packing of the per-process RCCL exchange (spacedrive_amd/shard.py) ----------

int sd_cas_exchange_pack_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint32_t* d_pos,
                             size_t n, uint64_t file0, uint32_t* d_rows, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n && (!d_keys || !d_pos || !d_rows)) return sd_fail(c, SD_CAS_EINVAL, "exchange_pack: null");
  if (file0 + n > (1ull << 32)) return sd_fail(c, SD_CAS_EINVAL, "exchange_pack: idx past u32");
  HIP_TRY(c, exch_pack(d_keys, d_pos, n, file0, d_rows, sd_pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_exchange_split_dev(sd_cas_ctx* c, const uint32_t* d_rows, size_t m, uint64_t* d_keys,
                              uint32_t* d_vals, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (m && (!d_rows || !d_keys || !d_vals)) return sd_fail(c, SD_CAS_EINVAL, "exchange_split: null");
  HIP_TRY(c, exch_split(d_rows, m, d_keys, d_vals, sd_pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_exchange_unpack_dev(sd_cas_ctx* c, const uint32_t* d_back, const uint32_t* d_pos,
                               size_t n, uint64_t* d_rep, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (n && (!d_back || !d_pos || !d_rep)) return sd_fail(c, SD_CAS_EINVAL, "exchange_unpack: null");
  HIP_TRY(c, exch_unpack(d_back, d_pos, n, d_rep, sd_pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_exchange_pack_fixed_dev(sd_cas_ctx* c, const uint64_t* d_keys, const uint32_t* d_pos,
                                   const uint64_t* d_counts, uint32_t G, uint64_t cap,
                                   uint64_t spill, uint64_t file0, uint32_t* d_rows,
                                   uint32_t* d_spill_rows, uint32_t* d_overflow, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (G == 0 || G > 1024 || cap == 0 || !d_counts || !d_rows || !d_overflow || (spill && !d_spill_rows))
    return sd_fail(c, SD_CAS_EINVAL, "exchange_pack_fixed: bad arguments");
  if (file0 >= (1ull << 32))  // file0 + every local position must fit in u32 (the caller checks n)
    return sd_fail(c, SD_CAS_EINVAL, "exchange_pack_fixed: idx past u32");
  HIP_TRY(c, exch_pack_fixed(d_keys, d_pos, d_counts, G, cap, spill, file0, d_rows, d_spill_rows,
                             d_overflow, sd_pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_exchange_split_fixed_dev(sd_cas_ctx* c, const uint32_t* d_rows, size_t m,
                                    uint64_t sentinel, uint64_t* d_keys, uint32_t* d_vals,
                                    uint64_t* d_sentinel_rows, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (m && (!d_rows || !d_keys || !d_vals || !d_sentinel_rows))
    return sd_fail(c, SD_CAS_EINVAL, "exchange_split_fixed: null");
  HIP_TRY(c, exch_split_fixed(d_rows, m, sentinel, d_keys, d_vals, d_sentinel_rows, sd_pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_exchange_unpack_fixed_dev(sd_cas_ctx* c, const uint32_t* d_back,
                                     const uint32_t* d_spill_back, const uint32_t* d_pos,
                                     const uint64_t* d_counts, uint32_t G, uint64_t cap,
                                     uint64_t spill, uint64_t* d_rep, void* stream) {
  if (!c) return SD_CAS_EINVAL;
  if (G == 0 || G > 1024 || cap == 0 || !d_back || !d_pos || !d_counts || !d_rep || (spill && !d_spill_back))
    return sd_fail(c, SD_CAS_EINVAL, "exchange_unpack_fixed: bad arguments");
  HIP_TRY(c, exch_unpack_fixed(d_back, d_spill_back, d_pos, d_counts, G, cap, spill, d_rep,
                               sd_pick(c, stream)));
  return SD_CAS_OK;
}

int sd_cas_copy_objects_dev(sd_cas_ctx* c, uint64_t* d_dst, void* stream) {
  if (!c || !d_dst) return SD_CAS_EINVAL;
  hipStream_t s = sd_pick(c, stream);
  const int k = c->region_obj_set;
  if (k >= 0) {  // the fused chain's last grouping: its region set's counter, after its tables
    HIP_TRY(c, hipStreamWaitEvent(s, c->region_done[k], 0));
    const uint64_t* obj = (const uint64_t*)((const char*)c->regions[k].p +
                                            sdcas::region_group_workspace_bytes(c->region_n[k]));
    HIP_TRY(c, hipMemcpyAsync(d_dst, obj, 8, hipMemcpyDeviceToDevice, s));
    // the set's next refill (its K1G zeroes this counter) must also wait for this copy
    HIP_TRY(c, hipEventRecord(c->region_done[k], s));
    return SD_CAS_OK;
  }
  HIP_TRY(c, sd_ws_acquire(c, s));
  HIP_TRY(c, hipMemcpyAsync(d_dst, c->d_scalar, 8, hipMemcpyDeviceToDevice, s));
  HIP_TRY(c, sd_ws_release(c, s));
  return SD_CAS_OK;
}

}  // extern "C"
