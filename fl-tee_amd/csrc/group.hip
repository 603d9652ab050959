// group.hip — one enclave id over several GPUs of one node, behind the
// unchanged ECALL ABI.
//
// The reference enclave is single-threaded; FL-TEE's only partitioning of the
// aggregation is alg 6's client batching inside the ECALL (lib.rs:498-573).  Here
// fltee_device_init_multi() returns an eid that spans W devices, and the ECALLs of
// that eid shard the work internally, so a Rust host that links this library gets
// the whole node through ecalls.rs as it stands:
//
//   dense baseline / non_oblivious / path_oram (every client uploads all d records,
//     serialize_dense): PARAMETER-RANGE sharding.  GPU r copies only its column slice
//     [p_r, p_r+1) of every client's ciphertext over its own PCIe link (a 2-D copy),
//     decrypts it with the counter offset of the slice, sums the n clients in order
//     (the single-GPU kernel on slice-local positions) and sends its averaged slice to
//     the root (RCCL).  Bit-identical to one GPU: each output is the same in-order sum.
//   advanced (alg 1): POSITION-RANGE sharding of the padded array (Option B): the
//     reference's bitonic network run distributed (range sorts; per stage two RCCL
//     all-to-alls transpose the rank bits into the range so its cross-range steps run
//     locally), one halo exchange for the fold, per-range oblivious compaction, and
//     ONE RCCL reduce (sum) of the W outputs on the root.  Bit-identical to one GPU.
//   nips19 (alg 2): the same distributed network with the keyed comparator (pairwise
//     range exchanges: the comparator reads the position); each range selects its
//     entries with idx < d in order, the lists are gathered to the root in range order
//     (= the global shuffled order) and the root runs the ordered fold.  Bit-identical.
//   optimized (alg 6): the batches are split over the GPUs; each GPU's batch sums are
//     sent to the root as rows, which adds them in batch order (lib.rs:564-573).
//     Bit-identical to one GPU.
//   sparse flat algorithms: the root alone (they take microseconds).
//
// Devices all distinct: RCCL over xGMI, one communicator per device
// (ncclCommInitAll), one stream per device, collectives as grouped send/recv and one
// ncclReduce.  All ranks on ONE device (the same id repeated): virtual ranks for the
// single-GPU tests, every range on one stream and the exchanges device copies.
//
// RCCL is opened on first use (dlopen, RTLD_LOCAL | RTLD_DEEPBIND), not linked: a host
// process may already hold another RCCL (PyTorch ships its own librccl.so), and two
// RCCLs resolving each other's symbols corrupt both.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "common.h"
#include "engine.h"
#include "group.h"

namespace fltee {

hipError_t launch_rows_accumulate(const float *mat, size_t n, size_t d, float coef, float *out,
                                  bool accumulate, hipStream_t s);

struct Rank {
    int dev = 0;
    hipStream_t s = nullptr;
    ncclComm_t comm = nullptr;
    Buffer cipher, rec, rk, out, chunk, spare, fold, fold_dst, cbuf, ctmp, lap, list, cnt, st;
    Buffer side, tot;  // advanced's fold: side records; its total, then the totals before it
};

struct Group {
    int W = 0;
    bool rccl = false;
    std::vector<Rank> r;
    Buffer rows;                    // root: W x d reduce rows (virtual ranks) / alg-6 batch rows
    uint32_t *host = nullptr;       // pinned readback words
};

struct RcclApi {
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, int,
                           ncclComm_t, hipStream_t);
    const char *(*GetErrorString)(ncclResult_t);
};

static const RcclApi *rccl() {
    static const RcclApi *api = [] () -> const RcclApi * {
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND))) break;
        if (!h) {
            std::fprintf(stderr, "[fltee] RCCL not found: %s\n", dlerror());
            return nullptr;
        }
        static RcclApi a;
        bool ok = true;
        auto get = [&](auto &fn, const char *sym) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, sym));
            ok = ok && fn;
        };
        get(a.CommInitAll, "ncclCommInitAll");
        get(a.CommDestroy, "ncclCommDestroy");
        get(a.GroupStart, "ncclGroupStart");
        get(a.GroupEnd, "ncclGroupEnd");
        get(a.Send, "ncclSend");
        get(a.Recv, "ncclRecv");
        get(a.Reduce, "ncclReduce");
        get(a.GetErrorString, "ncclGetErrorString");
        return ok ? &a : nullptr;
    }();
    return api;
}

static const char *nccl_err(ncclResult_t r) {
    return rccl() ? rccl()->GetErrorString(r) : "RCCL unavailable";
}

static void group_free(Group *G);

Group *group_create(const int *devs, int n, uint32_t *status) {
    *status = FLTEE_ERROR_INVALID_PARAMETER;
    if (!devs || n < 1 || n > 64 || (n & (n - 1))) return nullptr;  // ranges need a power of two
    bool all_same = true, distinct = true;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) {
            if (devs[i] != devs[j]) all_same = false;
            else distinct = false;
        }
    if (n == 1) all_same = false;  // one device: a one-rank RCCL communicator
    if (!all_same && !distinct) return nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) { *status = FLTEE_ERROR_UNEXPECTED; return nullptr; }
    for (int i = 0; i < n; ++i)
        if (devs[i] < 0 || devs[i] >= count) { *status = FLTEE_ERROR_UNEXPECTED; return nullptr; }
    Group *G = new Group;
    G->W = n;
    G->rccl = !all_same;
    G->r.resize(n);
    *status = FLTEE_ERROR_UNEXPECTED;
    for (int i = 0; i < n; ++i) {
        Rank &R = G->r[i];
        R.dev = devs[i];
        if (hipSetDevice(R.dev) != hipSuccess || !device_ctx(R.dev)) { group_free(G); return nullptr; }
        if (G->rccl || i == 0) {
            if (hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking) != hipSuccess) { group_free(G); return nullptr; }
        } else {
            R.s = G->r[0].s;  // virtual ranks share one stream
        }
    }
    if (G->rccl) {
        if (!rccl()) { group_free(G); return nullptr; }
        std::vector<ncclComm_t> comms(n);
        const ncclResult_t nr = rccl()->CommInitAll(comms.data(), n, devs);
        if (nr != ncclSuccess) {
            std::fprintf(stderr, "[fltee] ncclCommInitAll: %s\n", nccl_err(nr));
            group_free(G);
            return nullptr;
        }
        for (int i = 0; i < n; ++i) G->r[i].comm = comms[i];
    }
    (void)hipSetDevice(devs[0]);
    if (hipHostMalloc((void **)&G->host, 64 * 8, hipHostMallocDefault) != hipSuccess) {
        G->host = nullptr;
        group_free(G);
        return nullptr;
    }
    *status = FLTEE_SUCCESS;
    return G;
}

// Everything the group owns: per-rank buffers (they belong to the eid, not to the
// per-device scratch), the streams (virtual ranks share rank 0's), the communicators,
// the root's rows and the pinned readback words.
static void group_free(Group *G) {
    if (!G) return;
    for (size_t i = 0; i < G->r.size(); ++i) {
        Rank &R = G->r[i];
        if (hipSetDevice(R.dev) != hipSuccess) continue;
        if (R.s && (G->rccl || i == 0)) (void)fl_stream_sync(R.s);
        for (Buffer *b : {&R.cipher, &R.rec, &R.rk, &R.out, &R.chunk, &R.spare, &R.fold, &R.fold_dst,
                          &R.cbuf, &R.ctmp, &R.lap, &R.list, &R.cnt, &R.st})
            b->release();
        if (R.comm) (void)rccl()->CommDestroy(R.comm);
        R.comm = nullptr;
        if (R.s && (G->rccl || i == 0)) (void)hipStreamDestroy(R.s);
        R.s = nullptr;
    }
    if (!G->r.empty() && hipSetDevice(G->r[0].dev) == hipSuccess) {
        G->rows.release();
        if (G->host) (void)hipHostFree(G->host);
        G->host = nullptr;
    }
    delete G;
}

void group_destroy(Group *G) { group_free(G); }

int group_size(const Group *G) { return G ? G->W : 0; }
int group_root_device(const Group *G) { return G ? G->r[0].dev : -1; }
hipStream_t group_root_stream(const Group *G) { return G ? G->r[0].s : nullptr; }

static bool reserve_on(const Rank &R, Buffer &b, size_t bytes) {
    return hipSetDevice(R.dev) == hipSuccess && b.reserve(bytes);
}

static hipError_t sync_all(Group &G) {
    for (int i = 0; i < G.W; ++i) {
        if (!G.rccl && i) break;
        if (hipSetDevice(G.r[i].dev) != hipSuccess) return hipErrorInvalidDevice;
        const hipError_t e = fl_stream_sync(G.r[i].s);
        if (e != hipSuccess) return e;
    }
    (void)hipSetDevice(G.r[0].dev);
    return hipSuccess;
}

// ------------------------------------------------------------- transport ----
struct P2P {
    int src, dst;
    const void *sp;
    void *dp;
    size_t bytes;
};

// Every op moves `bytes` from rank src's buffer to rank dst's.  RCCL: one group of
// sends/receives on the ranks' streams (copies within a device are plain D2D
// copies); virtual ranks: device copies on the shared stream, in list order.
static hipError_t p2p(Group &G, const std::vector<P2P> &ops) {
    if (!G.rccl) {
        for (const P2P &o : ops) {
            if (!o.bytes || o.sp == o.dp) continue;
            const hipError_t e = fl_memcpy_async(o.dp, o.sp, o.bytes, hipMemcpyDeviceToDevice, G.r[0].s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    for (const P2P &o : ops) {  // local copies first (outside the RCCL group)
        if (!o.bytes || o.src != o.dst || o.sp == o.dp) continue;
        if (hipSetDevice(G.r[o.src].dev) != hipSuccess) return hipErrorInvalidDevice;
        const hipError_t e =
            fl_memcpy_async(o.dp, o.sp, o.bytes, hipMemcpyDeviceToDevice, G.r[o.src].s);
        if (e != hipSuccess) return e;
    }
    const RcclApi &nc = *rccl();
    ncclResult_t nr = nc.GroupStart();
    for (const P2P &o : ops) {
        if (nr != ncclSuccess) break;
        if (!o.bytes || o.src == o.dst) continue;
        if (trace_on()) trace_event("rccl_sendrecv", "", o.bytes, (uint64_t)o.src, (uint64_t)o.dst);
        nr = nc.Send(o.sp, o.bytes, ncclUint8, o.dst, G.r[o.src].comm, G.r[o.src].s);
        if (nr == ncclSuccess)
            nr = nc.Recv(o.dp, o.bytes, ncclUint8, o.src, G.r[o.dst].comm, G.r[o.dst].s);
    }
    const ncclResult_t ne = nc.GroupEnd();
    if (nr != ncclSuccess || ne != ncclSuccess) {
        std::fprintf(stderr, "[fltee] rccl p2p: %s\n", nccl_err(nr != ncclSuccess ? nr : ne));
        return hipErrorUnknown;
    }
    (void)hipSetDevice(G.r[0].dev);
    return hipSuccess;
}

// out_root[0, count) = sum over ranks of the ranks' `out` buffers (f32).  RCCL: one
// ncclReduce; virtual ranks: their outputs are rows of G.rows, summed in rank order.
// Used where exactly one rank holds each nonzero (+0.0 elsewhere): exact in any order.
static hipError_t reduce_to_root(Group &G, size_t count, float *out_root) {
    if (!G.rccl)
        return launch_rows_accumulate((const float *)G.rows.ptr, G.W, count, 1.0f, out_root, false,
                                      G.r[0].s);
    const RcclApi &nc = *rccl();
    if (trace_on()) trace_event("rccl_reduce", "", count * 4, (uint64_t)G.W, 0);
    ncclResult_t nr = nc.GroupStart();
    for (int i = 0; i < G.W && nr == ncclSuccess; ++i)
        nr = nc.Reduce(G.r[i].out.ptr, i == 0 ? (void *)out_root : nullptr, count, ncclFloat,
                       ncclSum, 0, G.r[i].comm, G.r[i].s);
    const ncclResult_t ne = nc.GroupEnd();
    if (nr != ncclSuccess || ne != ncclSuccess) {
        std::fprintf(stderr, "[fltee] rccl reduce: %s\n", nccl_err(nr != ncclSuccess ? nr : ne));
        return hipErrorUnknown;
    }
    return hipSuccess;
}

// the per-rank f32[count] output buffer (a row of G.rows for virtual ranks)
static float *rank_out(Group &G, int i, size_t count) {
    if (!G.rccl) {
        if (!reserve_on(G.r[0], G.rows, (size_t)G.W * count * 4)) return nullptr;
        return (float *)G.rows.ptr + (size_t)i * count;
    }
    if (!reserve_on(G.r[i], G.r[i].out, count * 4)) return nullptr;
    return (float *)G.r[i].out.ptr;
}

// ---------------------------------------------------------- small kernels ---
__global__ void fill_u64_kernel(uint64_t *p, size_t n, uint64_t v) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = v;
}
static hipError_t fill_pads(uint64_t *p, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    size_t b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    FLTEE_LAUNCH(fill_u64_kernel, dim3((unsigned)b), dim3(256), 0, s, p, n, (uint64_t)0xFFFFFFFFu);
    return hipGetLastError();
}

static uint32_t read_words(Group &G, const std::vector<const uint32_t *> &words,
                           std::vector<uint32_t> &vals) {
    vals.assign(words.size(), 0);
    for (size_t i = 0; i < words.size(); ++i) {
        const Rank &R = G.r[G.rccl ? i : 0];
        if (hipSetDevice(R.dev) != hipSuccess ||
            fl_memcpy_async(G.host + i, words[i], 4, hipMemcpyDeviceToHost, R.s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (sync_all(G) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    for (size_t i = 0; i < words.size(); ++i) vals[i] = G.host[i];
    return FLTEE_SUCCESS;
}

// records [lo, hi) of the root's array to every rank r (its range of positions) —
// virtual ranks just point into the root's array
static hipError_t scatter_records(Group &G, const uint64_t *root_rec, size_t nrec,
                                  const std::vector<size_t> &lo, const std::vector<size_t> &hi,
                                  std::vector<const uint64_t *> &rec_r) {
    rec_r.assign(G.W, nullptr);
    std::vector<P2P> ops;
    for (int i = 0; i < G.W; ++i) {
        const size_t a = lo[i] < nrec ? lo[i] : nrec, b = hi[i] < nrec ? hi[i] : nrec;
        if (!G.rccl || i == 0) {
            rec_r[i] = root_rec + a;
            continue;
        }
        if (!reserve_on(G.r[i], G.r[i].rec, (b - a) * 8 + 16)) return hipErrorOutOfMemory;
        rec_r[i] = (const uint64_t *)G.r[i].rec.ptr;
        ops.push_back({0, i, root_rec + a, G.r[i].rec.ptr, (b - a) * 8});
    }
    return p2p(G, ops);
}

// The records each rank needs: positions [lo[i], hi[i]) of the n*rpc client-major
// records.  From the host ciphertext (in.enc): every GPU copies the whole
// clients that cover its range over its own PCIe link (one host thread per GPU) and
// decrypts them itself; rec_r[i] points at position lo[i].  Otherwise from the root's
// decrypted records (scatter_records).  Virtual ranks take the per-GPU path too (all
// on one device), so the one-GPU tests cover its client ranges and offsets.
static uint32_t group_records(Group &G, const GroupInput &in, size_t n, size_t rpc,
                              const std::vector<size_t> &lo, const std::vector<size_t> &hi,
                              std::vector<const uint64_t *> &rec_r) {
    const size_t nrec = n * rpc;
    if (!in.enc) {
        if (!in.root_rec) return FLTEE_ERROR_UNEXPECTED;
        return scatter_records(G, in.root_rec, nrec, lo, hi, rec_r) == hipSuccess
                   ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
    }
    const int W = G.W;
    rec_r.assign(W, nullptr);
    std::vector<size_t> c_lo(W), c_hi(W);
    std::vector<uint32_t> errs(W, 0);
    for (int i = 0; i < W; ++i) {
        const size_t a = lo[i] < nrec ? lo[i] : nrec, b = hi[i] < nrec ? hi[i] : nrec;
        c_lo[i] = rpc ? a / rpc : 0;
        c_hi[i] = (rpc && b > a) ? (b + rpc - 1) / rpc : c_lo[i];
    }
    const auto t0 = std::chrono::steady_clock::now();
    auto load = [&](int i) {
        Rank &R = G.r[i];
        const size_t nc = c_hi[i] - c_lo[i];
        if (hipSetDevice(R.dev) != hipSuccess) { errs[i] = 1; return; }
        if (!R.cipher.reserve(nc * in.bpc + 16) || !R.rec.reserve(nc * rpc * 8 + 16) ||
            !R.rk.reserve(nc * 44 * 4 + 16)) { errs[i] = 3; return; }
        if (nc == 0) return;
        if (fl_memcpy_async(R.rk.ptr, in.rk + c_lo[i] * 44, nc * 44 * 4, hipMemcpyHostToDevice, R.s) != hipSuccess ||
            fl_memcpy_async(R.cipher.ptr, in.enc + c_lo[i] * in.bpc, nc * in.bpc, hipMemcpyHostToDevice,
                           R.s) != hipSuccess ||
            fl_stream_sync(R.s) != hipSuccess)
            errs[i] = 1;
    };
    std::vector<std::thread> th;
    for (int i = 0; i < W; ++i) th.emplace_back(load, i);
    for (auto &t : th) t.join();
    for (int i = 0; i < W; ++i)
        if (errs[i]) return errs[i] == 3 ? FLTEE_ERROR_OUT_OF_MEMORY : FLTEE_ERROR_UNEXPECTED;
    const auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < W; ++i) {
        Rank &R = G.r[i];
        const size_t nc = c_hi[i] - c_lo[i];
        rec_r[i] = (const uint64_t *)R.rec.ptr + (lo[i] < nrec ? lo[i] - c_lo[i] * rpc : 0);
        if (nc == 0) continue;
        if (hipSetDevice(R.dev) != hipSuccess ||
            launch_aes_ctr((const uint8_t *)R.cipher.ptr, nc, in.bpc, rpc, (const uint32_t *)R.rk.ptr,
                           (uint8_t *)R.rec.ptr, R.s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (sync_all(G) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    if (in.t_load) *in.t_load = std::chrono::duration<float>(t1 - t0).count();
    if (in.t_dec) *in.t_dec = std::chrono::duration<float>(std::chrono::steady_clock::now() - t1).count();
    return FLTEE_SUCCESS;
}

// ================================================================ dense =====
// Parameter-range shard of dense uploads, straight from the host ciphertext.
uint32_t group_dense_ecall(Group *Gp, const uint32_t *rk_host, size_t n, const uint8_t *enc,
                           size_t d, float coef, float *d_out_root, float *t_load, float *t_dec,
                           bool reject_order) {
    Group &G = *Gp;
    const int W = G.W;
    std::vector<size_t> p(W + 1);
    // multiples of 4: whole 16-B AES blocks, 16-B aligned output slices
    for (int i = 0; i <= W; ++i) p[i] = (d * (size_t)i / (size_t)W) & ~(size_t)3;
    p[W] = d;
    const size_t bpc = d * 8;
    std::vector<uint32_t> errs(W, 0);
    auto t0 = std::chrono::steady_clock::now();
    // one host thread per GPU: pageable H2D copies to different GPUs overlap only when
    // issued from different threads
    auto work = [&](int i) {
        Rank &R = G.r[i];
        const size_t dg = p[i + 1] - p[i];
        if (hipSetDevice(R.dev) != hipSuccess) { errs[i] = 1; return; }
        if (dg == 0) return;
        if (!R.cipher.reserve(n * dg * 8) || !R.rec.reserve(n * dg * 8) || !R.rk.reserve(n * 44 * 4) ||
            !R.st.reserve(64)) { errs[i] = 3; return; }
        if (fl_memset_async(R.st.ptr, 0, 4, R.s) != hipSuccess ||
            fl_memcpy_async(R.rk.ptr, rk_host, n * 44 * 4, hipMemcpyHostToDevice, R.s) != hipSuccess ||
            fl_memcpy2d_async(R.cipher.ptr, dg * 8, enc + p[i] * 8, bpc, dg * 8, n, hipMemcpyHostToDevice,
                             R.s) != hipSuccess) { errs[i] = 1; return; }
    };
    std::vector<std::thread> th;
    if (G.rccl && W > 1) {
        for (int i = 0; i < W; ++i) th.emplace_back(work, i);
        for (auto &t : th) t.join();
    } else {
        for (int i = 0; i < W; ++i) work(i);
    }
    for (int i = 0; i < W; ++i)
        if (errs[i]) return errs[i] == 3 ? FLTEE_ERROR_OUT_OF_MEMORY : FLTEE_ERROR_UNEXPECTED;
    if (sync_all(G) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    auto t1 = std::chrono::steady_clock::now();
    if (t_load) *t_load = std::chrono::duration<float>(t1 - t0).count();
    std::vector<P2P> gather;
    for (int i = 0; i < W; ++i) {
        Rank &R = G.r[i];
        const size_t dg = p[i + 1] - p[i];
        if (dg == 0) continue;
        if (hipSetDevice(R.dev) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
        float *o = G.rccl && i ? nullptr : d_out_root + p[i];
        if (!o) {
            if (!R.out.reserve(dg * 4)) return FLTEE_ERROR_OUT_OF_MEMORY;
            o = (float *)R.out.ptr;
            gather.push_back({i, 0, o, d_out_root + p[i], dg * 4});
        }
        if (launch_aes_ctr_slice((const uint8_t *)R.cipher.ptr, n, dg * 8, dg, (const uint32_t *)R.rk.ptr,
                                 (uint8_t *)R.rec.ptr, p[i] / 2, (uint32_t)p[i], R.s) != hipSuccess ||
            launch_dense_accumulate(R.rec.ptr, n, dg, coef, o, nullptr, false, (uint32_t *)R.st.ptr,
                                    R.s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (p2p(G, gather) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    std::vector<const uint32_t *> sw;
    for (int i = 0; i < W; ++i) sw.push_back((const uint32_t *)G.r[i].st.ptr);
    std::vector<uint32_t> st;
    if (read_words(G, sw, st)) return FLTEE_ERROR_UNEXPECTED;
    if (t_dec) *t_dec = std::chrono::duration<float>(std::chrono::steady_clock::now() - t1).count();
    for (uint32_t v : st)
        if (v & FLTEE_DEV_ERR_DENSE_ORDER)  // not dense: rejected, or the root's sparse rerun
            return reject_order ? FLTEE_ERROR_INVALID_PARAMETER : FLTEE_GROUP_FALLBACK;
    for (uint32_t v : st)
        if (v) return FLTEE_ERROR_UNEXPECTED;
    return FLTEE_SUCCESS;
}

// ===================================================== distributed network ==
// The reference network over M positions in W ranges of C (rank r: [r*C, (r+1)*C)):
// range sorts, then per stage the cross-range steps (transposed: two all-to-alls
// around local register passes, mode 0; pairwise: a swap with partner r ^ j/C per
// step) and the range merges — fltee/parallel.py distributed_network, on the ranks.
// valid: positions >= valid hold identical pads.  As in the single-GPU network, a stage
// leaves every aligned 2^stage block of pads alone unchanged: a range sort runs only on
// its live prefix (none at all for a range of pads), and a later stage skips the ranges
// at or past roundup(valid, 2^stage) — their pairwise partners lie in the same block,
// so both sides of a skipped exchange are skipped.  The transposed exchange mixes
// every range, so its stages skip nothing.  Public sizes only: still oblivious.
static hipError_t network(Group &G, std::vector<uint64_t *> &chunk, std::vector<uint64_t *> &spare,
                          size_t M, uint32_t mode, uint32_t key, bool transpose, size_t valid) {
    const int W = G.W;
    const size_t C = M / W;
    const uint32_t clog = log2_pow2(C), mlog = log2_pow2(M), wlog = log2_pow2(W);
    if (valid > M || !pad_skip_enabled()) valid = M;
    auto live_from = [&](uint32_t stage) -> size_t {  // ranges r with r*C >= this are pads alone
        const size_t blk = (size_t)1 << stage;
        const size_t b = (valid + blk - 1) / blk * blk;
        return b >= M ? M : b;
    };
    hipError_t e;
    for (int i = 0; i < W; ++i) {
        const size_t lo = (size_t)i * C;
        if (lo >= valid) continue;  // pads alone
        const size_t vl = valid - lo;
        if ((e = hipSetDevice(G.r[i].dev)) != hipSuccess) return e;
        if ((e = bitonic_sort_range(chunk[i], C, mode, key, (uint32_t)lo, G.r[i].s,
                                    vl >= C ? 0u : (uint32_t)vl)) != hipSuccess)
            return e;
    }
    const size_t b = C / W;
    for (uint32_t stage = clog + 1; stage <= mlog; ++stage) {
        if (transpose) {
            for (int pass = 0; pass < 2; ++pass) {
                std::vector<P2P> ops;
                for (int r = 0; r < W; ++r)
                    for (int q = 0; q < W; ++q)  // block q of range r -> block r of range q
                        ops.push_back({r, q, chunk[r] + q * b, spare[q] + r * b, b * 8});
                if ((e = p2p(G, ops)) != hipSuccess) return e;
                std::swap(chunk, spare);
                if (pass == 0)
                    for (int i = 0; i < W; ++i) {  // global bit `stage` = local bit stage - wlog
                        if ((e = hipSetDevice(G.r[i].dev)) != hipSuccess) return e;
                        if ((e = bitonic_steps_range(chunk[i], C, mode, key, stage - wlog,
                                                     stage - 1 - wlog, clog - wlog, 0u,
                                                     G.r[i].s)) != hipSuccess)
                            return e;
                    }
            }
        } else {
            const size_t sf = live_from(stage);
            for (int j = (int)stage - 1; j >= (int)clog; --j) {
                const int bit = 1 << (j - (int)clog);
                std::vector<P2P> ops;
                for (int r = 0; r < W; ++r)
                    if ((size_t)r * C < sf) ops.push_back({r ^ bit, r, chunk[r ^ bit], spare[r], C * 8});
                if ((e = p2p(G, ops)) != hipSuccess) return e;
                for (int r = 0; r < W; ++r) {
                    if ((size_t)r * C >= sf) continue;
                    if ((e = hipSetDevice(G.r[r].dev)) != hipSuccess) return e;
                    if ((e = bitonic_exchange(chunk[r], spare[r], C, (uint32_t)(r * C),
                                              (uint32_t)((r ^ bit) * C), mode, key, stage,
                                              (uint32_t)j, G.r[r].s)) != hipSuccess)
                        return e;
                }
            }
        }
        const size_t sf = transpose ? M : live_from(stage);
        for (int i = 0; i < W; ++i) {
            if ((size_t)i * C >= sf) continue;
            if ((e = hipSetDevice(G.r[i].dev)) != hipSuccess) return e;
            if ((e = bitonic_merge_range(chunk[i], C, mode, key, stage, (uint32_t)(i * C), G.r[i].s)) != hipSuccess)
                return e;
        }
    }
    return hipSuccess;
}

static bool reserve_chunks(Group &G, size_t C, std::vector<uint64_t *> &chunk,
                           std::vector<uint64_t *> &spare) {
    chunk.assign(G.W, nullptr);
    spare.assign(G.W, nullptr);
    for (int i = 0; i < G.W; ++i) {
        Rank &R = G.r[i];
        if (!reserve_on(R, R.chunk, C * 8) || !reserve_on(R, R.spare, C * 8)) return false;
        chunk[i] = (uint64_t *)R.chunk.ptr;
        spare[i] = (uint64_t *)R.spare.ptr;
    }
    return true;
}

// ============================================================= advanced =====
uint32_t group_advanced(Group *Gp, const GroupInput &in, size_t n, size_t k, size_t d,
                        float coef, float *d_out_root) {
    Group &G = *Gp;
    const int W = G.W;
    const size_t nrec = n * k, L = nrec + d, M = next_pow2_sz(L), C = M / W;
    if (C < (size_t)W * 16 || M > ((size_t)1 << 29)) return FLTEE_GROUP_FALLBACK;
    std::vector<uint64_t *> chunk, spare;
    if (!reserve_chunks(G, C, chunk, spare)) return FLTEE_ERROR_OUT_OF_MEMORY;
    std::vector<size_t> lo(W), hi(W);
    for (int i = 0; i < W; ++i) lo[i] = i * C, hi[i] = (i + 1) * C;
    std::vector<const uint64_t *> rec;
    if (uint32_t st = group_records(G, in, n, k, lo, hi, rec)) return st;
    for (int i = 0; i < W; ++i) {  // advanced.rs:116-142 on each range
        if (hipSetDevice(G.r[i].dev) != hipSuccess ||
            launch_advanced_init_range(rec[i], nrec, d, i * C, C, chunk[i], G.r[i].s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (network(G, chunk, spare, M, 0, 0, W > 1, n * k + d) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    // fold (advanced.rs:66-101) with the previous range's tail in front (the halo and the
    // record before it) and the next range's head behind, halo n; then the long-run patch
    // (k_fold.hip): every range's segmented total goes to the ranges after it (device to
    // device), which finish the runs begun before them.  Fixed cost: no status readback.
    const size_t fold_len = L;
    const size_t h = n;
    const size_t X = fold_context(h) + 16;  // context records in front of each range
    std::vector<float *> outs(W);
    {
        if (X > C) return FLTEE_GROUP_FALLBACK;
        const size_t m = X + C + 16;
        const size_t lanes = fold_lanes(C, fold_len, h, X, 1);
        std::vector<P2P> ops;
        for (int i = 0; i < W; ++i) {
            Rank &R = G.r[i];
            if (!reserve_on(R, R.fold, m * 8) || !reserve_on(R, R.fold_dst, m * 8) ||
                !reserve_on(R, R.side, fold_side_bytes(C, fold_len, h, X, 1) + 64) ||
                !reserve_on(R, R.tot, (size_t)(W + 1) * sizeof(FoldAgg)))
                return FLTEE_ERROR_OUT_OF_MEMORY;
            uint64_t *f = (uint64_t *)R.fold.ptr;
            ops.push_back({i, i, chunk[i], f + X, C * 8});
            if (i > 0) ops.push_back({i - 1, i, chunk[i - 1] + C - X, f, X * 8});
            if (i < W - 1) ops.push_back({i + 1, i, chunk[i + 1], f + X + C, 16 * 8});
            if ((i == 0 && fill_pads(f, X, R.s) != hipSuccess) ||
                (i == W - 1 && fill_pads(f + X + C, 16, R.s) != hipSuccess))
                return FLTEE_ERROR_UNEXPECTED;
        }
        if (p2p(G, ops) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
        // tot[0] = this range's total, tot[1 + j] = range j's (j < i)
        for (int i = 0; i < W; ++i) {
            Rank &R = G.r[i];
            if (hipSetDevice(R.dev) != hipSuccess ||
                launch_fold_range((const uint64_t *)R.fold.ptr, (uint64_t *)R.fold_dst.ptr, m, X, X + C,
                                  (long long)(i * C) - (long long)X, fold_len, h, (FoldSide *)R.side.ptr,
                                  R.s) != hipSuccess ||
                launch_fold_range_total((const FoldSide *)R.side.ptr, lanes, (FoldAgg *)R.tot.ptr,
                                        R.s) != hipSuccess)
                return FLTEE_ERROR_UNEXPECTED;
        }
        std::vector<P2P> tops;
        for (int i = 0; i < W; ++i)
            for (int j = 0; j < i; ++j)
                tops.push_back({j, i, G.r[j].tot.ptr, (FoldAgg *)G.r[i].tot.ptr + 1 + j, sizeof(FoldAgg)});
        if (p2p(G, tops) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
        for (int i = 0; i < W; ++i) {
            Rank &R = G.r[i];
            if (hipSetDevice(R.dev) != hipSuccess ||
                launch_fold_range_patch((uint64_t *)R.fold_dst.ptr, C, X, (long long)(i * C) - (long long)X,
                                        fold_len, h, (const FoldSide *)R.side.ptr,
                                        (const FoldAgg *)R.tot.ptr + 1, (size_t)i, R.s) != hipSuccess)
                return FLTEE_ERROR_UNEXPECTED;
        }
    }
    for (int i = 0; i < W; ++i) {  // advanced.rs:106-111 + :32-34: each range's representatives
        Rank &R = G.r[i];
        float *o = rank_out(G, i, d);
        if (!o || !reserve_on(R, R.cbuf, (d + C) * 8) || !reserve_on(R, R.ctmp, (d + C) * 8))
            return FLTEE_ERROR_OUT_OF_MEMORY;
        outs[i] = o;
        if (launch_compact_offset((const uint64_t *)R.fold_dst.ptr + X, C, d,
                                  (uint64_t *)R.cbuf.ptr, (uint64_t *)R.ctmp.ptr, 1.0f, o, R.s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (hipSetDevice(G.r[0].dev) != hipSuccess || reduce_to_root(G, d, d_out_root) != hipSuccess ||
        (coef != 1.0f && launch_scale(d_out_root, d, coef, G.r[0].s) != hipSuccess))
        return FLTEE_ERROR_UNEXPECTED;
    return sync_all(G) == hipSuccess ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
}

// =============================================================== nips19 =====
uint32_t group_nips19(Group *Gp, DeviceCtx *root, const GroupInput &in, size_t n, size_t k,
                      size_t k_req, size_t d, uint64_t seed, float coef, float *d_out_root) {
    Group &G = *Gp;
    const int W = G.W;
    const float T = nips19_threshold(d, k_req, n);
    const size_t tf = !(T > 0.0f) ? 0 : (size_t)T;
    const size_t nrec = n * k, L = nrec + d * tf, M = next_pow2_sz(L), C = M / W;
    if (C < 64 || M > ((size_t)1 << 29) || d == 0) return FLTEE_GROUP_FALLBACK;
    const uint32_t key = (uint32_t)(seed ^ (seed >> 32));  // the shuffle key of aggregate()
    std::vector<uint64_t *> chunk, spare;
    if (!reserve_chunks(G, C, chunk, spare)) return FLTEE_ERROR_OUT_OF_MEMORY;
    std::vector<size_t> lo(W), hi(W);
    for (int i = 0; i < W; ++i) lo[i] = i * C, hi[i] = (i + 1) * C;
    std::vector<const uint64_t *> rec;
    if (uint32_t st = group_records(G, in, n, k, lo, hi, rec)) return st;
    for (int i = 0; i < W; ++i) {  // every rank draws the same counts (counter-based Philox)
        Rank &R = G.r[i];
        if (!reserve_on(R, R.lap, d * 4)) return FLTEE_ERROR_OUT_OF_MEMORY;
        if (launch_laplace_r(d, k_req, T, seed, (uint32_t *)R.lap.ptr, R.s) != hipSuccess ||
            launch_nips19_build_range(rec[i], nrec, (const uint32_t *)R.lap.ptr, d, tf, i * C, C,
                                      chunk[i], R.s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (network(G, chunk, spare, M, 2, key, false, nrec + d * tf) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    // safe_aggregate (common.rs:25-35): every range selects its idx < d entries in order;
    // the lists, concatenated in range order, are the shuffled array's in position order
    const size_t nb = select_tiles(C);
    std::vector<const uint32_t *> tw;
    for (int i = 0; i < W; ++i) {
        Rank &R = G.r[i];
        if (!reserve_on(R, R.cnt, (2 * nb + 2) * 4)) return FLTEE_ERROR_OUT_OF_MEMORY;
        uint32_t *cnt = (uint32_t *)R.cnt.ptr;
        if (launch_select_count(chunk[i], C, d, cnt, cnt + nb + 1, R.s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
        tw.push_back(cnt + nb + 1 + nb);
    }
    std::vector<uint32_t> tot;
    if (read_words(G, tw, tot)) return FLTEE_ERROR_UNEXPECTED;
    size_t lc = 0;
    std::vector<size_t> off(W);
    for (int i = 0; i < W; ++i) off[i] = lc, lc += tot[i];
    if (hipSetDevice(G.r[0].dev) != hipSuccess || !root->ws_sel.reserve(lc * 8 + 8))
        return FLTEE_ERROR_OUT_OF_MEMORY;
    uint64_t *list = (uint64_t *)root->ws_sel.ptr;
    std::vector<P2P> ops;
    for (int i = 0; i < W; ++i) {
        Rank &R = G.r[i];
        uint64_t *dst = list + off[i];
        if (G.rccl && i) {
            if (!reserve_on(R, R.list, tot[i] * 8 + 8)) return FLTEE_ERROR_OUT_OF_MEMORY;
            dst = (uint64_t *)R.list.ptr;
            ops.push_back({i, 0, dst, list + off[i], (size_t)tot[i] * 8});
        }
        const uint32_t *cnt = (const uint32_t *)R.cnt.ptr;
        if (tot[i] && launch_select_write(chunk[i], C, d, cnt + nb + 1, dst, R.s) != hipSuccess)
            return FLTEE_ERROR_UNEXPECTED;
    }
    if (p2p(G, ops) != hipSuccess || hipSetDevice(G.r[0].dev) != hipSuccess ||
        !G.r[0].st.reserve(64) ||
        ordered_from_list(root, list, lc, d, coef, d_out_root, false, (uint32_t *)G.r[0].st.ptr,
                          G.r[0].s) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    return sync_all(G) == hipSuccess ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
}

// ========================================================= optimized (alg 6) =
uint32_t group_optimized(Group *Gp, const GroupInput &in, size_t n, size_t k, size_t d,
                         size_t batch, float coef, float *d_out_root, size_t halo) {
    Group &G = *Gp;
    const int W = G.W;
    if (batch == 0) return FLTEE_ERROR_INVALID_PARAMETER;
    const size_t nbt = (n + batch - 1) / batch;  // batches, lib.rs:498-572
    if (!reserve_on(G.r[0], G.rows, nbt * d * 4 + 16)) return FLTEE_ERROR_OUT_OF_MEMORY;
    float *rows = (float *)G.rows.ptr;
    std::vector<size_t> b0(W), b1(W), lo(W), hi(W);
    for (int i = 0; i < W; ++i) {
        b0[i] = nbt * i / W, b1[i] = nbt * (i + 1) / W;
        lo[i] = b0[i] * batch * k;
        hi[i] = (b1[i] * batch < n ? b1[i] * batch : n) * k;
    }
    std::vector<const uint64_t *> rec;
    if (uint32_t st = group_records(G, in, n, k, lo, hi, rec)) return st;
    const size_t h = halo;  // halo n: bit for bit up to n + 1 entries a run, re-associated beyond
    {
        std::vector<P2P> ops;
        std::vector<const uint32_t *> sw;
        for (int i = 0; i < W; ++i) {
            Rank &R = G.r[i];
            const size_t nb_i = b1[i] - b0[i];
            if (!reserve_on(R, R.st, 64)) return FLTEE_ERROR_OUT_OF_MEMORY;
            float *myrows = rows + b0[i] * d;
            if (G.rccl && i) {
                if (!reserve_on(R, R.out, nb_i * d * 4 + 16)) return FLTEE_ERROR_OUT_OF_MEMORY;
                myrows = (float *)R.out.ptr;
                ops.push_back({i, 0, myrows, rows + b0[i] * d, nb_i * d * 4});
            }
            if (fl_memset_async(R.st.ptr, 0, 4, R.s) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
            for (size_t b = b0[i]; b < b1[i]; ++b) {
                const size_t c0 = b * batch, nb = (c0 + batch < n ? batch : n - c0);
                if (advanced_batch(rec[i] + (c0 * k - lo[i]), nb, k, d, h, myrows + (b - b0[i]) * d,
                                   (uint32_t *)R.st.ptr, R.s) != hipSuccess)
                    return FLTEE_ERROR_UNEXPECTED;
            }
            sw.push_back((const uint32_t *)R.st.ptr);
        }
        (void)sw;  // (the folds finish runs of any length: no status to read back)
        if (p2p(G, ops) != hipSuccess) return FLTEE_ERROR_UNEXPECTED;
    }
    // lib.rs:564-573: global[i] += batch_sum[i] in batch order, then x 1f32/n
    if (hipSetDevice(G.r[0].dev) != hipSuccess ||
        launch_rows_accumulate(rows, nbt, d, coef, d_out_root, false, G.r[0].s) != hipSuccess)
        return FLTEE_ERROR_UNEXPECTED;
    return sync_all(G) == hipSuccess ? FLTEE_SUCCESS : FLTEE_ERROR_UNEXPECTED;
}

}  // namespace fltee

namespace fltee {
bool group_splits_host_copy(const Group *G) { return G && G->W > 1; }
}  // namespace fltee
