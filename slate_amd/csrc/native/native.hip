// Native (Python-free) host runtime and drivers of slate_amd: see
// include/slate_amd/slate_native.hh.
//
// The step loops are the same MI355X designs as the Python drivers
// (slate_amd/models/chol.py, lu.py, blas3.py), written against the HIP
// runtime and the transport of native_comm.hip directly:
//   * one process per GPU; world communicator from a TCP-bootstrapped RCCL
//     unique id (or the host-staged transport); row / column communicators
//     by split, each driven from ONE stream (collectives keep one order on
//     every rank and add no hardware queue);
//   * a high-priority panel stream, a low-priority update stream and a comm
//     stream per process, dependencies as HIP events, no host
//     synchronisation inside a factorization (info values are read once at
//     the end);
//   * every flop on the hand-written gfx950 kernels of csrc/hip (potrf_mc /
//     potrf_lds tile Cholesky, trsm_rlt, the persistent LU panel and the
//     distributed LU column step, the MFMA GEMM with block-cyclic masks);
//   * four precisions (s, d, c, z), as the reference instantiates every
//     routine (src/potrf.cc:285-303).
// Reference call stacks: src/potrf.cc:22-210, src/getrf.cc:22-244,
// src/gemmC.cc:39-202, src/work/work_trsm.cc:102-265 (SLATE's OpenMP task
// DAGs over MPI).
#include <algorithm>
#include <array>
#include <atomic>
#include <limits>
#include <functional>
#include <map>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <tuple>
#include <vector>

#include <hip/hip_ext.h>

#include "../hip/kernels.hpp"
#include "../hip/launchers.hpp"
#include "../hip/workspace.hpp"
#include "native_rt.hpp"

namespace slate_amd {
namespace native {

// ------------------------------------------------------------ runtime
Runtime& rt() {
    static Runtime r;
    return r;
}

static int env_int(const char* k, int def) {
    const char* v = std::getenv(k);
    return v && *v ? std::atoi(v) : def;
}

static void initialize_rt();

void initialize() {
    if (rt().up) return;
    initialize_rt();
    static std::once_flag traced;
    std::call_once(traced, [] { trace_rt::auto_start(); });
}

static void initialize_rt() {
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    if (R.up) return;
    R.rank = env_int("RANK", 0);
    R.size = env_int("WORLD_SIZE", 1);
    R.local = env_int("LOCAL_RANK", 0);
    int ndev = 1;
    NHIP(hipGetDeviceCount(&ndev));
    R.device = env_int("SLATE_AMD_NATIVE_DEVICE", ndev > 0 ? R.local % ndev : 0);
    NHIP(hipSetDevice(R.device));
    int lo = 0, hi = 0;
    NHIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    NHIP(hipStreamCreateWithFlags(&R.main, hipStreamNonBlocking));
    NHIP(hipStreamCreateWithPriority(&R.panel, hipStreamNonBlocking, hi));
    NHIP(hipStreamCreateWithPriority(&R.update, hipStreamNonBlocking, lo));
    // one rank: no collectives, so no comm stream of its own -- the box has
    // 4 hardware queues, and a 5th stream (the CU-masked update stream is
    // created next to the plain one) could put the high-priority panel
    // stream on the queue of the bulk GEMMs (ADVICE r4 for the Python path)
    if (R.size > 1) NHIP(hipStreamCreateWithPriority(&R.comm, hipStreamNonBlocking, hi));
    else R.comm = R.main;
    // diagnostics: SLATE_AMD_NATIVE_SERIAL=1 issues everything on one stream
    if (env_int("SLATE_AMD_NATIVE_SERIAL", 0)) R.panel = R.update = R.comm = R.main;
    const size_t lw = slate_hip::getrf_work_bytes();
    NHIP(hipMalloc(&R.lu_work, lw));
    NHIP(hipMemset(R.lu_work, 0, lw));
    const size_t qw = std::max<size_t>(64, slate_hip::geqrf_work_bytes());
    NHIP(hipMalloc(&R.qr_work, qw));
    NHIP(hipMemset(R.qr_work, 0, qw));
    transport_init(R.rank, R.size);
    R.up = true;
}

void finalize() {
    if (rt().up) trace_rt::auto_finish();
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    if (!R.up) return;
    (void)hipDeviceSynchronize();
    if (R.size > 1 && world_comm()) {
        // no rank unmaps a mailbox a peer's kernel may still post into
        bool peers = false;
        for (auto& g : R.grids) peers = peers || (g.second && g.second->colpeer);
        if (peers) {
            Scratch d(sizeof(i64), R.main);
            dzero(d.p, sizeof(i64), R.main);
            world_comm()->allreduce(d.p, 1, DT::I64, 's', R.main);
            NHIP(hipStreamSynchronize(R.main));
        }
    }
    R.grids.clear();
    transport_finalize();
    (void)hipFree(R.lu_work);
    (void)hipFree(R.qr_work);
    slate_hip::dev_trim();              // cached scratch blocks back to the driver
    std::vector<hipStream_t> ss{R.main, R.panel, R.update, R.comm};
    for (auto& kv : R.parked) if (kv.second) ss.push_back(kv.second);
    R.parked.clear();
    R.update_res = 0;
    std::sort(ss.begin(), ss.end());
    ss.erase(std::unique(ss.begin(), ss.end()), ss.end());
    for (hipStream_t s : ss) (void)hipStreamDestroy(s);
    R.up = false;
}

// The update streams of each reservation are created once per process and
// kept (parked) on one rank: re-creating the masked stream per
// factorization cost 3 % of a native dgetrf, and a fifth stream next to a
// comm stream of its own put the panel stream on the bulk GEMMs' hardware
// queue (the box has 4): dgetrf n = 32768 36.5 -> 43.3 TF/s with the comm
// stream aliased to main on one rank (profiles/r6/getrf_reservation_keep.txt).
void set_update_reservation(int cus) {
    Runtime& R = rt();
    if (cus == R.update_res || R.update == R.main) return;
    static int ncu = 0;
    if (!ncu) {
        hipDeviceProp_t pr;
        NHIP(hipGetDeviceProperties(&pr, R.device));
        ncu = pr.multiProcessorCount;
    }
    if (!(cus > 0 && cus < ncu)) cus = 0;
    if (cus == R.update_res) return;
    NHIP(hipStreamSynchronize(R.update));
    // one rank (comm = main): park the old stream -- 4 streams in all.  With a
    // comm stream of its own a parked 5th stream could share a hardware
    // queue with the panel stream: destroy it instead
    if (R.size == 1) R.parked[R.update_res] = R.update;
    else NHIP(hipStreamDestroy(R.update));
    auto it = R.parked.find(cus);
    if (it != R.parked.end() && it->second) {
        R.update = it->second;
        R.parked.erase(it);
    } else if (cus > 0) {
        // the first mask bits map round-robin to the 8 XCDs: the reserved CUs
        // are spread evenly (same mask as the Python driver, streams.py)
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int b = cus; b < ncu; ++b) mask[b / 32] |= 1u << (b % 32);
        NHIP(hipExtStreamCreateWithCUMask(&R.update, (uint32_t)mask.size(), mask.data()));
    } else {
        int lo = 0, hi = 0;
        NHIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        NHIP(hipStreamCreateWithPriority(&R.update, hipStreamNonBlocking, lo));
    }
    R.update_res = cus;
}

PeerBox::~PeerBox() {
    (void)hipDeviceSynchronize();
    for (void* p : opened) slate_hip::lu_peer_close(p);
    if (own) slate_hip::lu_peer_free(own);
    (void)hipFree(mbox_d);
    (void)hipFree(part);
    (void)hipFree(err);
}

PeerBox* peer_box(Comm* c, std::unique_ptr<PeerBox>& slot, hipStream_t s) {
    if (slot && slot->dead)
        throw Error("native getrf: this grid's peer mailboxes timed out earlier (sequence tags no longer agree "
                    "across ranks); build a new grid to continue");
    if (slot) return slot.get();
    const char* e = std::getenv("SLATE_AMD_LU_PEER");
    if ((e && e[0] == '0') || !c || c->size < 2 || c->size > slate_hip::lu_peer_max_p()) return nullptr;
    auto pb = std::make_unique<PeerBox>();
    char h[64];
    pb->own = slate_hip::lu_peer_alloc(slate_hip::lu_peer_mailbox_bytes(), h);
    // the 64-byte handles travel once over the communicator itself
    Scratch hs(64 * (size_t)(c->size + 1), s);
    upload(static_cast<char*>(hs.p) + 64 * c->size, h, 64, s);
    c->allgather(static_cast<char*>(hs.p) + 64 * c->size, hs.p, 64, s);
    std::vector<char> all((size_t)64 * c->size);
    NHIP(hipMemcpyAsync(all.data(), hs.p, all.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    std::vector<unsigned long long> ptrs((size_t)c->size);
    for (int r = 0; r < c->size; ++r) {
        if (r == c->rank) ptrs[r] = (unsigned long long)(uintptr_t)pb->own;
        else {
            void* q = slate_hip::lu_peer_open(all.data() + 64 * (size_t)r);
            pb->opened.push_back(q);
            ptrs[r] = (unsigned long long)(uintptr_t)q;
        }
    }
    NHIP(hipMalloc(&pb->mbox_d, ptrs.size() * sizeof(unsigned long long)));
    NHIP(hipMemcpy(pb->mbox_d, ptrs.data(), ptrs.size() * sizeof(unsigned long long), hipMemcpyHostToDevice));
    NHIP(hipMalloc(&pb->part, slate_hip::lu_peer_part_bytes()));
    NHIP(hipMemset(pb->part, 0, slate_hip::lu_peer_part_bytes()));
    NHIP(hipMalloc(&pb->err, sizeof(unsigned long long)));
    NHIP(hipMemset(pb->err, 0, sizeof(unsigned long long)));
    NHIP(hipDeviceSynchronize());
    // every member has mapped every mailbox before any kernel posts into one
    Scratch d(sizeof(i64), s);
    dzero(d.p, sizeof(i64), s);
    c->allreduce(d.p, 1, DT::I64, 's', s);
    NHIP(hipStreamSynchronize(s));
    slot = std::move(pb);
    return slot.get();
}

namespace {
// RAII: the LU trailing update leaves the persistent panel's CUs free for the
// duration of one factorization, then the update stream is unmasked again
struct UpdateReservation {
    explicit UpdateReservation(int cus) { set_update_reservation(cus); }
    ~UpdateReservation() {
        try { set_update_reservation(0); } catch (...) {}
    }
};
}  // namespace

int rank() { initialize(); return rt().rank; }
int size() { initialize(); return rt().size; }
const char* version() { return "slate_amd-native 2026.10.0"; }
const char* transport() { initialize(); return transport_name(); }

void barrier() {
    initialize();
    Runtime& R = rt();
    NHIP(hipDeviceSynchronize());
    if (R.size == 1) return;
    Scratch d(sizeof(i64), R.main);
    dzero(d.p, sizeof(i64), R.main);
    world_comm()->allreduce(d.p, 1, DT::I64, 's', R.main);
    NHIP(hipStreamSynchronize(R.main));
}

double allreduce_max(double v) {
    initialize();
    Runtime& R = rt();
    if (R.size == 1) return v;
    Scratch d(sizeof(double), R.main);
    upload(d.p, &v, sizeof(double), R.main);
    world_comm()->allreduce(d.p, 1, DT::F64, 'M', R.main);
    NHIP(hipMemcpyAsync(&v, d.p, sizeof(double), hipMemcpyDeviceToHost, R.main));
    NHIP(hipStreamSynchronize(R.main));
    return v;
}

// row / column communicators of a p x q column-major grid (collective:
// every rank creates the grids in the same order)
GridComms* grid_comms(int p, int q) {
    Runtime& R = rt();
    if (p * q != R.size)
        throw Error("grid " + std::to_string(p) + "x" + std::to_string(q) + " does not match " +
                    std::to_string(R.size) + " ranks");
    auto key = std::make_pair(p, q);
    auto it = R.grids.find(key);
    if (it != R.grids.end()) return it->second.get();
    auto g = std::make_unique<GridComms>();
    g->p = p;
    g->q = q;
    g->pr = R.rank % p;
    g->pc = R.rank / p;
    if (R.size > 1) {
        g->row = world_comm()->split(g->pr, g->pc);
        g->col = world_comm()->split(g->pc, g->pr);
        // the update stream's twin of `col` (an RCCL communicator is driven
        // from one stream: the TSQR trailing all-reduces run beside the panel's)
        if (p > 1) g->colu = world_comm()->split(g->pc, g->pr);
    }
    GridComms* out = g.get();
    R.grids[key] = std::move(g);
    return out;
}

// ------------------------------------------------------------ storage
template <typename T>
Matrix<T>::Matrix(int64_t m, int64_t n, int64_t nb, int p, int q) {
    initialize();
    if (m < 0 || n < 0 || nb <= 0 || p <= 0 || q <= 0) throw Error("Matrix: bad dimensions");
    auto s = std::make_shared<Storage>();
    s->m = m; s->n = n; s->nb = nb; s->p = p; s->q = q;
    s->gc = grid_comms(p, q);
    s->pr = s->gc->pr; s->pc = s->gc->pc;
    s->mloc = numroc(m, nb, s->pr, p);
    s->nloc = numroc(n, nb, s->pc, q);
    s->lld = std::max<i64>(1, (s->mloc + 15) / 16 * 16);
    s->esize = sizeof(T);
    const size_t bytes = (size_t)s->lld * std::max<i64>(s->nloc, 1) * sizeof(T);
    NHIP(hipMalloc(&s->buf, bytes));
    dzero(s->buf, bytes, rt().main);
    NHIP(hipStreamSynchronize(rt().main));
    s_ = s;
}
template <typename T>
Matrix<T> Matrix<T>::from_device(T* d_local, int64_t lld, int64_t m, int64_t n, int64_t nb, int p, int q) {
    initialize();
    if (m < 0 || n < 0 || nb <= 0 || p <= 0 || q <= 0) throw Error("Matrix::from_device: bad dimensions");
    auto s = std::make_shared<Storage>();
    s->m = m; s->n = n; s->nb = nb; s->p = p; s->q = q;
    s->gc = grid_comms(p, q);
    s->pr = s->gc->pr; s->pc = s->gc->pc;
    s->mloc = numroc(m, nb, s->pr, p);
    s->nloc = numroc(n, nb, s->pc, q);
    if (lld < std::max<i64>(1, s->mloc)) throw Error("Matrix::from_device: lld < local rows");
    if (!d_local && s->mloc && s->nloc) throw Error("Matrix::from_device: null buffer");
    s->lld = lld;
    s->esize = sizeof(T);
    s->buf = d_local;
    s->owns = false;
    Matrix<T> M;
    M.s_ = s;
    return M;
}

template <typename T>
Matrix<T> Matrix<T>::sub(int64_t i0, int64_t i1, int64_t j0, int64_t j1) const {
    (void)storage();           // plain matrices only (a view throws)
    const Storage& P = *s_;
    const i64 mt = (P.m + P.nb - 1) / P.nb, nt = (P.n + P.nb - 1) / P.nb;
    if (i0 < 0 || j0 < 0 || i1 > mt || j1 > nt || i0 > i1 || j0 > j1)
        throw Error("Matrix::sub: tile range outside the matrix");
    if (i0 % P.p || j0 % P.q)
        throw Error("Matrix::sub: the first tile row (column) must be a multiple of p (q)");
    auto s = std::make_shared<Storage>();
    s->m = std::min(i1 * P.nb, P.m) - i0 * P.nb;
    s->n = std::min(j1 * P.nb, P.n) - j0 * P.nb;
    s->nb = P.nb; s->p = P.p; s->q = P.q; s->pr = P.pr; s->pc = P.pc; s->gc = P.gc;
    s->mloc = numroc(s->m, P.nb, P.pr, P.p);
    s->nloc = numroc(s->n, P.nb, P.pc, P.q);
    s->lld = P.lld;
    s->esize = P.esize;
    s->buf = static_cast<char*>(P.buf) + ((i0 / P.p) * P.nb + (j0 / P.q) * P.nb * P.lld) * (i64)P.esize;
    s->owns = false;
    s->parent = s_;
    Matrix<T> M;
    M.s_ = s;
    return M;
}

template <typename T> int64_t Matrix<T>::m() const { return op_ == Op::NoTrans ? s_->m : s_->n; }
template <typename T> int64_t Matrix<T>::n() const { return op_ == Op::NoTrans ? s_->n : s_->m; }
template <typename T>
std::shared_ptr<Storage> Matrix<T>::storage() const {
    if (op_ != Op::NoTrans)
        throw Error("native: this routine does not take a transposed view (materialise it with copy())");
    return s_;
}
template <typename T>
void Matrix<T>::apply_op(Op o) {
    op_ = compose_op<T>(o, op_);
}
template <typename T> int64_t Matrix<T>::nb() const { return s_->nb; }
template <typename T> int Matrix<T>::p() const { return s_->p; }
template <typename T> int Matrix<T>::q() const { return s_->q; }
template <typename T> int64_t Matrix<T>::mloc() const { return s_->mloc; }
template <typename T> int64_t Matrix<T>::nloc() const { return s_->nloc; }
template <typename T> int64_t Matrix<T>::lld() const { return s_->lld; }
template <typename T> T* Matrix<T>::data() { return static_cast<T*>(s_->buf); }
template <typename T> const T* Matrix<T>::data() const { return static_cast<const T*>(s_->buf); }

template <typename T>
void Matrix<T>::generate(Gen kind, uint64_t seed) {
    (void)storage();           // plain matrices only (a view throws)
    Storage& s = *s_;
    slate_hip::matgen<K<T>>((int)kind, seed, s.mloc, s.nloc, kp(data()), s.lld, s.m, s.n, s.nb, s.p, s.pr, s.nb, s.q,
                            s.pc, 0, 0, 1.0, rt().main);
    NHIP(hipStreamSynchronize(rt().main));
}

// host <-> device transfers go through a contiguous staging buffer and the
// gecopy kernel (no pitched hipMemcpy2D: see copy2d below)
template <typename T>
void Matrix<T>::from_local_host(const T* Aloc, int64_t ld) {
    (void)storage();           // plain matrices only (a view throws)
    const Storage& s = *s_;
    Runtime& R = rt();
    if (!s.mloc || !s.nloc) return;
    std::vector<T> h((size_t)s.mloc * s.nloc);
    for (i64 j = 0; j < s.nloc; ++j)
        std::memcpy(h.data() + j * s.mloc, Aloc + j * ld, sizeof(T) * s.mloc);
    Scratch stg(h.size() * sizeof(T), R.main);
    upload(stg.p, h.data(), h.size() * sizeof(T), R.main);
    slate_hip::gecopy<K<T>, K<T>>('G', 'N', s.mloc, s.nloc, kp(stg.as<T>()), s.mloc, kp(static_cast<T*>(s.buf)),
                                  s.lld, R.main);
    NHIP(hipStreamSynchronize(R.main));
}

template <typename T>
void Matrix<T>::to_local_host(T* Aloc, int64_t ld) const {
    (void)storage();           // plain matrices only (a view throws)
    const Storage& s = *s_;
    Runtime& R = rt();
    NHIP(hipDeviceSynchronize());
    if (!s.mloc || !s.nloc) return;
    std::vector<T> h((size_t)s.mloc * s.nloc);
    Scratch stg(h.size() * sizeof(T), R.main);
    slate_hip::gecopy<K<T>, K<T>>('G', 'N', s.mloc, s.nloc, kp(static_cast<const T*>(s.buf)), s.lld,
                                  kp(stg.as<T>()), s.mloc, R.main);
    NHIP(hipMemcpyAsync(h.data(), stg.p, h.size() * sizeof(T), hipMemcpyDeviceToHost, R.main));
    NHIP(hipStreamSynchronize(R.main));
    for (i64 j = 0; j < s.nloc; ++j)
        std::memcpy(Aloc + j * ld, h.data() + j * s.mloc, sizeof(T) * s.mloc);
}

// (a view's rows are a strided window of its parent's buffer: every transfer
// goes through a contiguous mloc x nloc staging block)
template <typename T>
void Matrix<T>::from_host(const T* A, int64_t lda) {
    (void)storage();           // plain matrices only (a view throws)
    Storage& s = *s_;
    std::vector<T> loc((size_t)std::max<i64>(s.mloc, 1) * std::max<i64>(s.nloc, 1), T(0));
    for (i64 lj = 0; lj < s.nloc; ++lj) {
        const i64 gj = l2g(lj, s.nb, s.q, s.pc);
        for (i64 li = 0; li < s.mloc; ++li) loc[li + lj * s.mloc] = A[l2g(li, s.nb, s.p, s.pr) + gj * lda];
    }
    from_local_host(loc.data(), std::max<i64>(s.mloc, 1));
}

// every rank gets the whole matrix: ONE all-gather of the local blocks
// (padded to the largest local block), each rank scatters them on the host
template <typename T>
void Matrix<T>::to_host(T* A, int64_t lda) const {
    (void)storage();           // plain matrices only (a view throws)
    const Storage& s = *s_;
    Runtime& R = rt();
    NHIP(hipDeviceSynchronize());
    if (R.size == 1) {
        to_local_host(A, lda);
        return;
    }
    i64 mx_m = 0, mx_n = 0;
    for (int r = 0; r < s.p; ++r) mx_m = std::max(mx_m, numroc(s.m, s.nb, r, s.p));
    for (int c = 0; c < s.q; ++c) mx_n = std::max(mx_n, numroc(s.n, s.nb, c, s.q));
    const size_t blk = (size_t)std::max<i64>(mx_m, 1) * std::max<i64>(mx_n, 1) * sizeof(T);
    Scratch mine(blk, R.main), all(blk * R.size, R.main);
    if (s.mloc && s.nloc)
        slate_hip::gecopy<K<T>, K<T>>('G', 'N', s.mloc, s.nloc, kp(static_cast<const T*>(s.buf)), s.lld,
                                      kp(mine.as<T>()), std::max<i64>(mx_m, 1), R.main);
    world_comm()->allgather(mine.p, all.p, blk, R.main);
    std::vector<T> h(blk / sizeof(T) * R.size);
    NHIP(hipMemcpyAsync(h.data(), all.p, h.size() * sizeof(T), hipMemcpyDeviceToHost, R.main));
    NHIP(hipStreamSynchronize(R.main));
    const i64 ldb = std::max<i64>(mx_m, 1);
    for (int r = 0; r < R.size; ++r) {
        const int pr = r % s.p, pc = r / s.p;
        const i64 ml = numroc(s.m, s.nb, pr, s.p), nl = numroc(s.n, s.nb, pc, s.q);
        const T* b = h.data() + (size_t)r * (blk / sizeof(T));
        for (i64 lj = 0; lj < nl; ++lj) {
            const i64 gj = l2g(lj, s.nb, s.q, pc);
            for (i64 li = 0; li < ml; ++li) A[l2g(li, s.nb, s.p, pr) + gj * lda] = b[li + lj * ldb];
        }
    }
}

// ------------------------------------------------------------ helpers
namespace {


int64_t read_infos(const i64* d, i64 nt, hipStream_t s, i64 nb) {
    std::vector<i64> h((size_t)std::max<i64>(nt, 1));
    NHIP(hipMemcpyAsync(h.data(), d, h.size() * sizeof(i64), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    for (i64 t = 0; t < nt; ++t)
        if (h[t] > 0) return t * nb + h[t];
    return 0;
}

int64_t reduce_info(int64_t info) {
    Runtime& R = rt();
    if (R.size == 1) return info;
    const i64 big = (i64)1 << 62;
    Scratch d(sizeof(i64), R.main);
    i64 v = info > 0 ? info : big;
    upload(d.p, &v, sizeof(i64), R.main);
    world_comm()->allreduce(d.p, 1, DT::I64, 'm', R.main);
    NHIP(hipMemcpyAsync(&v, d.p, sizeof(i64), hipMemcpyDeviceToHost, R.main));
    NHIP(hipStreamSynchronize(R.main));
    return v >= big ? 0 : v;
}

// Lcol plan of one step (Python: models/_panels.py _rows_plan): for each
// process row r the local rows (relative to the local start of tile tfirst)
// it contributes, then where each needed tile's rows land, in tile order
struct ColPlan {
    std::vector<i64> off, cnt;      // per r: offset into idx, count
    i64 order_off = 0, order_cnt = 0, tot = 0;
};

ColPlan rows_plan(std::vector<i64>& flat, i64 m, i64 nb, int p, int q, int pc, i64 tfirst, i64 tend, i64 cols_from) {
    auto mb = [&](i64 j) { return std::min(nb, m - j * nb); };
    std::vector<i64> need;
    for (i64 j = cols_from; j < tend; ++j)
        if (j % q == pc) need.push_back(j);
    ColPlan P;
    P.off.assign(p, 0);
    P.cnt.assign(p, 0);
    std::vector<i64> base(p, 0), start(need.size(), 0);
    i64 pos = 0;
    for (int r = 0; r < p; ++r) {
        const i64 base_r = tiles_before(tfirst, p, r) * nb;
        P.off[r] = (i64)flat.size();
        base[r] = pos;
        i64 cur = 0;
        for (size_t t = 0; t < need.size(); ++t) {
            const i64 j = need[t];
            if (j % p != r) continue;
            const i64 lj = (j / p) * nb - base_r;
            start[t] = cur;
            for (i64 e = 0; e < mb(j); ++e) flat.push_back(lj + e);
            cur += mb(j);
        }
        P.cnt[r] = cur;
        pos += cur;
    }
    P.tot = pos;
    P.order_off = (i64)flat.size();
    for (size_t t = 0; t < need.size(); ++t) {
        const int r = (int)(need[t] % p);
        for (i64 e = 0; e < mb(need[t]); ++e) flat.push_back(base[r] + start[t] + e);
    }
    P.order_cnt = (i64)flat.size() - P.order_off;
    return P;
}

// Lcol (cnt x kb, contiguous) = the panel rows of this rank's local columns
// of the plan's tile range, from Prow (this process row's panel rows); the
// column broadcasts go on stream s (the column communicator's stream)
template <typename T>
void assemble_cols(const ColPlan& P, const i64* idx, const T* Prow, i64 ldp, i64 kb, GridComms* gc, T* Lcol,
                   hipStream_t s, Comm* col = nullptr) {
    if (!col) col = gc->col.get();
    if (P.tot == 0) return;
    Scratch R((size_t)P.tot * kb * sizeof(T), s);
    i64 pos = 0;
    for (int r = 0; r < gc->p; ++r) {
        const i64 cnt = P.cnt[r];
        if (cnt) {
            Scratch tmp((size_t)cnt * kb * sizeof(T), s);
            if (gc->pr == r)
                slate_hip::permute_rows_gather<K<T>>(cnt, kb, kp(Prow), ldp, kp(tmp.as<T>()), cnt, idx + P.off[r], s);
            if (gc->p > 1) col->bcast(tmp.p, (size_t)cnt * kb * sizeof(T), r, s);
            copy2d(R.as<T>() + pos, P.tot, tmp.as<T>(), cnt, cnt, kb, s);
        }
        pos += cnt;
    }
    slate_hip::permute_rows_gather<K<T>>(P.order_cnt, kb, kp(R.as<T>()), P.tot, kp(Lcol), P.order_cnt,
                                         idx + P.order_off, s);
}

// diagnostics (SLATE_AMD_NATIVE_DEBUG_SUMS=1): synchronise s and print the sum
// of |x| over an m x n block
template <typename T>
void dbg_sum(const char* tag, i64 t, const T* A, i64 ld, i64 m, i64 n, hipStream_t s) {
    static const bool on = env_int("SLATE_AMD_NATIVE_DEBUG_SUMS", 0) != 0;
    if (!on) return;
    NHIP(hipStreamSynchronize(s));
    double acc = 0;
    if (m > 0 && n > 0) {
        std::vector<T> h((size_t)ld * n);
        NHIP(hipMemcpy(h.data(), A, sizeof(T) * ((size_t)ld * (n - 1) + m), hipMemcpyDeviceToHost));
        for (i64 j = 0; j < n; ++j)
            for (i64 i = 0; i < m; ++i) acc += std::abs(h[i + j * ld]);
    }
    // the same block read by a KERNEL (one-norm column sums, genorm) -- a
    // copy engine reads memory, a kernel may read stale cache lines
    double kacc = 0;
    if constexpr (std::is_same<T, double>::value) {
        if (m > 0 && n > 0) {
            double* d = nullptr;
            NHIP(hipMalloc(&d, sizeof(double) * (n + m)));
            NHIP(hipMemset(d, 0, sizeof(double) * (n + m)));
            slate_hip::genorm<double, double>('1', 'G', 'N', 0, m, n, A, ld, d, s);
            std::vector<double> h2((size_t)(n + m));
            NHIP(hipStreamSynchronize(s));
            NHIP(hipMemcpy(h2.data(), d, sizeof(double) * (n + m), hipMemcpyDeviceToHost));
            NHIP(hipFree(d));
            for (i64 j = 0; j < n; ++j) kacc += h2[j];
        }
    }
    std::fprintf(stderr, "TRACE r%d t=%lld %s %lldx%lld %.17g kernel %.17g\n", rt().rank, (long long)t, tag,
                 (long long)m, (long long)n, acc, kacc);
}

// tile Cholesky / panel solve: the tuned fp64 kernels, the generic ones else
template <typename T>
void potrf_tile_k(i64 n, T* A, i64 lda, i64* info, hipStream_t s) {
    if constexpr (std::is_same<T, double>::value)
        if (slate_hip::potrf_fast((int)n, A, lda, info, 0, s)) return;
    slate_hip::potrf_tile<K<T>>('L', (int)n, kp(A), lda, info, s);
}
template <typename T>
void trsm_rlc(i64 m, i64 n, const T* L, i64 ldl, T* B, i64 ldb, hipStream_t s) {   // B = B L^{-H}
    if (m <= 0) return;
    slate_hip::trsm<K<T>>('R', 'L', ctrans<T>(), 'N', m, n, kv(T(1)), kp(L), ldl, kp(B), ldb, s);
}

}  // namespace

// ------------------------------------------------------------ potrf
// One rank owning the whole matrix: trailing update per GROUP of 2 tiles
// (K = 2 nb on the MFMA GEMM), lookahead in groups (chol.py
// _potrf_1x1_grouped).
template <typename T>
static void potrf_1x1(T* A, i64 lda, i64 n, i64 nb, int la, i64* infos) {
    Runtime& R = rt();
    hipStream_t ps = R.panel, us = R.update;
    const i64 nt = (n + nb - 1) / nb;
    const i64 G = 2;
    const char ct = ctrans<T>();
    auto off = [&](i64 t) { return std::min(t * nb, n); };
    const i64 ng = (nt + G - 1) / G;
    auto gstart = [&](i64 gi) { return gi < ng ? off(gi * G) : n; };
    std::vector<std::unique_ptr<Event>> ev_tr(ng);
    join(R.main, ps);
    join(R.main, us);
    for (i64 gi = 0; gi < ng; ++gi) {
        const i64 c0 = gstart(gi), c2 = gstart(gi + 1);
        const i64 tfirst = gi * G, tlast = std::min(nt, tfirst + G);
        if (gi - la - 1 >= 0) ev_tr[gi - la - 1]->wait(ps);
        {
        NTRACE("potrf::panel", ps);
        for (i64 u = tfirst; u < tlast; ++u) {
            const i64 cu = off(u), cu1 = off(u + 1);
            if (cu > c0) {
                // the group's earlier panels -> column u (rows >= cu)
                slate_hip::TriMask mk = lower_mask(nb, 1, 0, 1, 0, cu, cu);
                gemm_k<T>('N', ct, n - cu, cu1 - cu, cu - c0, T(-1), A + cu + c0 * lda, lda, A + cu + c0 * lda, lda,
                          T(1), A + cu + cu * lda, lda, ps, &mk);
            }
            potrf_tile_k<T>(cu1 - cu, A + cu + cu * lda, lda, infos + u, ps);
            if (n > cu1) trsm_rlc<T>(n - cu1, cu1 - cu, A + cu + cu * lda, lda, A + cu1 + cu * lda, lda, ps);
        }
        }
        // P = A[c0:n, c0:c2]; update columns [lo, hi) (rows >= lo) on stream s
        auto update = [&](i64 lo, i64 hi, hipStream_t s) {
            if (hi <= lo) return;
            slate_hip::TriMask mk = lower_mask(nb, 1, 0, 1, 0, lo, lo);
            gemm_k<T>('N', ct, n - lo, hi - lo, c2 - c0, T(-1), A + lo + c0 * lda, lda, A + lo + c0 * lda, lda, T(1),
                      A + lo + lo * lda, lda, s, &mk);
        };
        const i64 la_end = gstart(gi + 1 + la);
        if (gi >= 1 && la > 0) ev_tr[gi - 1]->wait(ps);
        {
            NTRACE("potrf::lookahead", ps);
            update(c2, la_end, ps);
        }
        Event ev_panel;
        ev_panel.record(ps);
        ev_panel.wait(us);
        NTRACE("potrf::update", us);
        const i64 nx_end = std::max(gstart(gi + 2 + la), la_end);
        update(la_end, nx_end, us);
        ev_tr[gi] = std::make_unique<Event>();
        ev_tr[gi]->record(us);
        update(nx_end, n, us);
    }
    join(ps, R.main);
    join(us, R.main);
}

// p x q grid (chol.py _potrf_lower): panel stream = tile potrf, column bcast
// of the diagonal tile, trsm, then the TILE-GRANULAR row broadcast of the
// panel (SLATE listBcastMT, potrf.cc:122-132): chunk 0 = the first tile row,
// then chunks of 16 tile rows, on the comm stream (the row communicator's
// stream) while the panel stream runs each chunk's lookahead GEMM as it
// lands; column gathers of the lookahead's transposed operands (column
// communicator, panel stream); update stream = the trailing transposed
// rows (second column communicator, q > 1) and the trailing GEMMs.
template <typename T>
static void potrf_grid(Storage& S, int la, i64* infos) {
    Runtime& R = rt();
    GridComms* gc = S.gc;
    const int p = S.p, q = S.q, pr = S.pr, pc = S.pc;
    const i64 nb = S.nb, n = S.n, lld = S.lld;
    const char ct = ctrans<T>();
    T* buf = static_cast<T*>(S.buf);
    const i64 nt = (n + nb - 1) / nb;
    const i64 lr_end = S.mloc, lc_end = S.nloc;
    const i64 chunk_rows = nb * std::max(1, env_int("SLATE_AMD_POTRF_CHUNK", 16));
    hipStream_t ps = R.panel, us = R.update, cs = R.comm;
    // plans (host, then one upload)
    std::vector<i64> flat;
    std::vector<std::pair<ColPlan, ColPlan>> plans((size_t)nt);
    for (i64 t = 0; t < nt; ++t) {
        const i64 e = std::min(t + 1 + la, nt);
        plans[t].first = rows_plan(flat, n, nb, p, q, pc, t + 1, e, t + 1);
        plans[t].second = rows_plan(flat, n, nb, p, q, pc, t + 1, nt, e);
    }
    if (flat.empty()) flat.push_back(0);
    Scratch idx(flat.size() * sizeof(i64), ps);
    upload(idx.p, flat.data(), flat.size() * sizeof(i64), ps);
    join(R.main, ps);
    join(R.main, us);
    join(R.main, cs);
    std::vector<std::unique_ptr<Event>> ev_tr((size_t)nt), ev_used((size_t)nt);
    // per-step operand buffers shared by the comm, panel and update streams:
    // a ring of NR sets; set t % NR is rewritten at step t only after the
    // update stream has finished step t - NR (explicit events -- no reliance
    // on the stream-ordered allocator's cross-stream reuse rules)
    const int NR = la + 3;
    std::vector<std::unique_ptr<Scratch>> ring_p, ring_a, ring_c;
    for (int r = 0; r < NR; ++r) {
        ring_p.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(lr_end, 1) * nb * sizeof(T), ps));
        ring_a.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(lc_end, 1) * nb * sizeof(T), ps));
        ring_c.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(lc_end, 1) * nb * sizeof(T), ps));
    }
    for (i64 t = 0; t < nt; ++t) {
        const i64 g = t;
        if (t >= NR) {
            ev_used[t - NR]->wait(ps);
            ev_used[t - NR]->wait(cs);
        }
        const i64 kb = std::min(nb, n - g * nb);
        const i64 lrg = tiles_before(g, p, pr) * nb, lcg = tiles_before(g, q, pc) * nb;
        const i64 lr1 = std::min(tiles_before(g + 1, p, pr) * nb, lr_end);
        const i64 lc1 = std::min(tiles_before(g + 1, q, pc) * nb, lc_end);
        const bool own_col = (g % q) == pc, own_diag = own_col && (g % p) == pr;
        if (t - la - 1 >= 0) ev_tr[t - la - 1]->wait(ps);
        std::unique_ptr<trace_rt::Scope> sp_panel(trace_rt::g_on ? new trace_rt::Scope("potrf::panel", ps) : nullptr);
        if (own_diag) dbg_sum("diag_in", t, buf + lrg + lcg * lld, lld, kb, kb, ps);
        if (own_diag) potrf_tile_k<T>(kb, buf + lrg + lcg * lld, lld, infos + t, ps);
        if (own_diag) dbg_sum("diag_out", t, buf + lrg + lcg * lld, lld, kb, kb, ps);
        const i64 nrow = lr_end - lr1;
        if (own_col) {
            const T* D = buf + lrg + lcg * lld;
            i64 ldd = lld;
            Scratch Dt(p > 1 ? (size_t)kb * kb * sizeof(T) : 0, ps);
            if (p > 1) {
                if (own_diag) copy2d(Dt.as<T>(), kb, buf + lrg + lcg * lld, lld, kb, kb, ps);
                gc->col->bcast(Dt.p, (size_t)kb * kb * sizeof(T), (int)(g % p), ps);
                D = Dt.as<T>();
                ldd = kb;
            }
            dbg_sum("D", t, D, ldd, kb, kb, ps);
            dbg_sum("panel_in", t, buf + lr1 + lcg * lld, lld, nrow, kb, ps);
            if (nrow) trsm_rlc<T>(nrow, kb, D, ldd, buf + lr1 + lcg * lld, lld, ps);
            dbg_sum("panel_out", t, buf + lr1 + lcg * lld, lld, nrow, kb, ps);
            if (env_int("SLATE_AMD_NATIVE_DEBUG_SUMS", 0) && nrow)
                dbg_sum("Winv", t, static_cast<double*>(slate_hip::workspace(ps, sizeof(double) * 1024, slate_hip::WS_C)),
                        1024, 1024, 1, ps);
        }
        sp_panel.reset();
        // panel -> row (Prow: nrow x kb, contiguous), tile-granular chunks
        Scratch* Prow = ring_p[t % NR].get();
        const T* P = buf + lr1 + lcg * lld;
        i64 ldp = lld;
        // chunk 0 holds every lookahead tile row this process row owns
        const i64 first_rows = std::max(nb, std::min(tiles_before(g + 1 + la, p, pr) * nb, lr_end) - lr1);
        std::vector<std::pair<i64, i64>> chunks;
        for (i64 a = 0; a < nrow;) {
            const i64 b = std::min(nrow, a + (a == 0 ? first_rows : chunk_rows));
            chunks.push_back({a, b});
            a = b;
        }
        std::vector<std::unique_ptr<Event>> landed(chunks.size());
        if (q > 1) {
            P = Prow->as<T>();
            ldp = std::max<i64>(nrow, 1);
            Event src;
            src.record(ps);                          // trsm done
            src.wait(cs);
            NTRACE("potrf::bcast", cs);
            for (size_t ci = 0; ci < chunks.size(); ++ci) {
                const i64 a = chunks[ci].first, b = chunks[ci].second;
                auto cb = std::make_unique<Scratch>((size_t)(b - a) * kb * sizeof(T), cs);
                if (own_col) copy2d(cb->as<T>(), b - a, buf + lr1 + a + lcg * lld, lld, b - a, kb, cs);
                gc->row->bcast(cb->p, (size_t)(b - a) * kb * sizeof(T), (int)(g % q), cs);
                copy2d(Prow->as<T>() + a, ldp, cb->as<T>(), b - a, b - a, kb, cs);
                landed[ci] = std::make_unique<Event>();
                landed[ci]->record(cs);
            }
        }
        auto land = [&](size_t ci) { if (q > 1) landed[ci]->wait(ps); };
        if (!chunks.empty()) land(0);
        std::unique_ptr<trace_rt::Scope> sp_la(trace_rt::g_on ? new trace_rt::Scope("potrf::lookahead", ps) : nullptr);
        // transposed operands: lookahead tiles (in chunk 0), then the rest
        const ColPlan& A1 = plans[t].first;
        const ColPlan& A2 = plans[t].second;
        Scratch* Lla = ring_a[t % NR].get();
        Scratch* Lcol = ring_c[t % NR].get();
        const i64* d_idx = idx.as<i64>();
        const T* La;
        i64 lda_la;
        if (p > 1 || q > 1) {
            assemble_cols<T>(A1, d_idx, P, ldp, kb, gc, Lla->as<T>(), ps);
            La = Lla->as<T>();
            lda_la = std::max<i64>(A1.order_cnt, 1);
        } else {
            La = P;
            lda_la = ldp;
        }
        const i64 lc_la = std::min(tiles_before(g + 1 + la, q, pc) * nb, lc_end);
        dbg_sum("La", t, La, lda_la, lc_la - lc1, kb, ps);
        if (t >= 1 && la > 0) ev_tr[t - 1]->wait(ps);
        for (size_t ci = 0; ci < chunks.size(); ++ci) {
            if (ci) land(ci);
            const i64 a = chunks[ci].first, b = chunks[ci].second;
            if (lc_la > lc1) {
                slate_hip::TriMask mk = lower_mask(nb, p, pr, q, pc, lr1 + a, lc1);
                gemm_k<T>('N', ct, b - a, lc_la - lc1, kb, T(-1), P + a, ldp, La, lda_la, T(1),
                          buf + lr1 + a + lc1 * lld, lld, ps, &mk);
            }
        }
        sp_la.reset();
        dbg_sum("la_out", t, buf + lr1 + lc1 * lld, lld, nrow, lc_la - lc1, ps);
        const T* Lc;
        i64 ldlc, loff;
        // q > 1: the trailing transposed rows are gathered from the UPDATE
        // stream over the second column communicator (chol.py, same choice;
        // SLATE_AMD_POTRF_LCOL_U=0 keeps them on the panel stream)
        static const bool lcol_u_env = env_int("SLATE_AMD_POTRF_LCOL_U", 1) != 0;
        const bool lcol_u = lcol_u_env && q > 1 && (p == 1 || gc->colu);
        Event ev_panel;
        if (lcol_u) {
            ev_panel.record(ps);
            ev_panel.wait(us);
        }
        if (p > 1 || q > 1) {
            if (lcol_u)
                assemble_cols<T>(A2, d_idx, P, ldp, kb, gc, Lcol->as<T>(), us, p > 1 ? gc->colu.get() : nullptr);
            else
                assemble_cols<T>(A2, d_idx, P, ldp, kb, gc, Lcol->as<T>(), ps);
            Lc = Lcol->as<T>();
            ldlc = std::max<i64>(A2.order_cnt, 1);
            loff = lc_la;
        } else {
            Lc = P;
            ldlc = ldp;
            loff = lc1;
        }
        if (!lcol_u) {
            ev_panel.record(ps);
            ev_panel.wait(us);
        }
        const i64 lc_nx = std::max(std::min(tiles_before(g + 2 + la, q, pc) * nb, lc_end), lc_la);
        NTRACE("potrf::update", us);
        for (int part = 0; part < 2; ++part) {
            const i64 c0 = part == 0 ? lc_la : lc_nx, c1 = part == 0 ? lc_nx : lc_end;
            if (c1 > c0 && nrow) {
                slate_hip::TriMask mk = lower_mask(nb, p, pr, q, pc, lr1, c0);
                gemm_k<T>('N', ct, nrow, c1 - c0, kb, T(-1), P, ldp, Lc + (c0 - loff), ldlc, T(1),
                          buf + lr1 + c0 * lld, lld, us, &mk);
            }
            if (part == 0) {
                ev_tr[t] = std::make_unique<Event>();
                ev_tr[t]->record(us);
            }
        }
        ev_used[t] = std::make_unique<Event>();
        ev_used[t]->record(us);
    }
    join(ps, R.main);
    join(us, R.main);
    join(cs, R.main);
    for (auto* v : {&ring_p, &ring_a, &ring_c})
        for (auto& x : *v) x->s = R.main;       // freed after every stream joined main
    idx.s = R.main;
}

template <typename T>
int64_t potrf(HermitianMatrix<T>& A, const Options& opts) {
    if (A.uplo() != Uplo::Lower) throw Error("native potrf: Lower storage only (use the conjugate transpose)");
    NTRACE("potrf", nullptr);
    Storage& S = *A.storage();
    Runtime& R = rt();
    const i64 nt = (S.n + S.nb - 1) / S.nb;
    const int la = std::max(0, opts.lookahead);
    Scratch infos(sizeof(i64) * std::max<i64>(nt, 1), R.main);
    dzero(infos.p, sizeof(i64) * std::max<i64>(nt, 1), R.main);
    if (S.p == 1 && S.q == 1 && nt > 2)
        potrf_1x1<T>(static_cast<T*>(S.buf), S.lld, S.n, S.nb, la, infos.as<i64>());
    else
        potrf_grid<T>(S, la, infos.as<i64>());
    const int64_t info = read_infos(infos.as<i64>(), nt, R.main, S.nb);
    return reduce_info(info);
}

// ------------------------------------------------------------ distributed trsm
// B = op(A)^{-1} B, Side Left, A the uplo triangle (SLATE work::trsm,
// src/work/work_trsm.cc:102-265, as a tile-step loop): per step k (forward
// for Lower/NoTrans, backward for Upper/NoTrans)
//   diagonal tile A_kk -> process row k%p (row comm); that row solves its
//   local columns of B_k; X_k -> every process row (column comm); panel
//   A(:, k) -> every process column (row comm); B_i -= A_ik X_k locally.
// ConjTrans of a Lower A is a backward Upper solve on A^H, materialised by
// one tile redistribution (p2p) first.
template <typename T>
static void transpose_tiles(const Storage& L, Storage& U, char ct);

// tri: the right-hand side is triangular in tile granularity and stays so
// (an identity solved into an inverse factor): 1 = only rhs tile columns
// <= k are touched at step k (Lower), 2 = only those >= k (Upper) -- n^3/3
// flops for L^{-1} instead of n^3
template <typename T>
static void trsm_left(char uplo, char diag, T alpha, const Storage& SA, Storage& SB, int tri = 0) {
    Runtime& R = rt();
    GridComms* gc = SB.gc;
    const int p = SB.p, q = SB.q, pr = SB.pr, pc = SB.pc;
    const i64 nb = SA.nb, n = SA.n, nrhs_all = SB.nloc;
    const T* A = static_cast<const T*>(SA.buf);
    T* B0 = static_cast<T*>(SB.buf);
    const i64 lda = SA.lld, ldb = SB.lld;
    const i64 nt = (n + nb - 1) / nb;
    hipStream_t s = R.main;
    if (alpha != T(1) && SB.mloc && nrhs_all) slate_hip::gescale<K<T>>('G', SB.mloc, nrhs_all, kv(alpha), kp(B0), ldb, s);
    const bool lower = uplo == 'L';
    for (i64 st = 0; st < nt; ++st) {
        const i64 k = lower ? st : nt - 1 - st;
        const i64 kb = std::min(nb, n - k * nb);
        const int rk = (int)(k % p), ck = (int)(k % q);
        const i64 lrk = tiles_before(k, p, pr) * nb, lck = tiles_before(k, q, pc) * nb;
        const i64 c0 = tri == 2 ? std::min(tiles_before(k, q, pc) * nb, nrhs_all) : 0;
        const i64 c1 = tri == 1 ? std::min(tiles_before(k + 1, q, pc) * nb, nrhs_all) : nrhs_all;
        const i64 nrhs_loc = std::max<i64>(c1 - c0, 0);
        T* B = B0 + c0 * ldb;
        // diagonal tile to process row rk
        Scratch D((size_t)kb * kb * sizeof(T), s);
        if (pr == rk) {
            if (pc == ck) copy2d(D.as<T>(), kb, A + lrk + lck * lda, lda, kb, kb, s);
            if (q > 1) gc->row->bcast(D.p, (size_t)kb * kb * sizeof(T), ck, s);
            if (nrhs_loc)
                slate_hip::trsm<K<T>>('L', uplo, 'N', diag, kb, nrhs_loc, kv(T(1)), kp(D.as<T>()), kb,
                                      kp(B + lrk), ldb, s);
        }
        // X_k to every process row
        Scratch X((size_t)kb * std::max<i64>(nrhs_loc, 1) * sizeof(T), s);
        if (pr == rk) copy2d(X.as<T>(), kb, B + lrk, ldb, kb, nrhs_loc, s);
        if (p > 1 && nrhs_loc) gc->col->bcast(X.p, (size_t)kb * nrhs_loc * sizeof(T), rk, s);
        // panel A(rows after / before k, k) of this process row
        const i64 r0 = lower ? std::min(tiles_before(k + 1, p, pr) * nb, SA.mloc) : 0;
        const i64 r1 = lower ? SA.mloc : std::min(tiles_before(k, p, pr) * nb, SA.mloc);
        const i64 nr = r1 - r0;
        if (nr <= 0) continue;
        Scratch Pn((size_t)nr * kb * sizeof(T), s);
        if (pc == ck) copy2d(Pn.as<T>(), nr, A + r0 + lck * lda, lda, nr, kb, s);
        if (q > 1) gc->row->bcast(Pn.p, (size_t)nr * kb * sizeof(T), ck, s);
        if (nrhs_loc)
            gemm_k<T>('N', 'N', nr, nrhs_loc, kb, T(-1), Pn.as<T>(), nr, X.as<T>(), kb, T(1), B + r0, ldb, s);
    }
    NHIP(hipStreamSynchronize(s));
}

// B = op(A)^{-1} B with op(A) = A^T (tr 'T') or A^H (tr 'C'), on the stored
// triangle -- no transposed copy of A.  Column-oriented ("left-looking")
// substitution: op(A)'s row k is A's column k, so per step k (backward for
// Lower, forward for Upper)
//   column k of A beyond the diagonal -> every process column (row comm);
//   W = A(beyond, k)^op B(beyond) locally (the rows beyond k already hold
//   their final X), summed over the process column (one nb x nrhs
//   all-reduce); process row k%p: B_k -= W, B_k = op(A_kk)^{-1} B_k.
// Per step O(local rows x nb) extra memory.  Reference: the transposed view
// of src/work/work_trsm.cc:102-265 (its tileBcast then fetches A(k, i)).
template <typename T>
static void trsm_left_t(char uplo, char diag, char tr, T alpha, const Storage& SA, Storage& SB) {
    Runtime& R = rt();
    GridComms* gc = SB.gc;
    const int p = SB.p, q = SB.q, pr = SB.pr, pc = SB.pc;
    const i64 nb = SA.nb, n = SA.n, nrhs_loc = SB.nloc;
    const T* A = static_cast<const T*>(SA.buf);
    T* B = static_cast<T*>(SB.buf);
    const i64 lda = SA.lld, ldb = SB.lld;
    const i64 nt = (n + nb - 1) / nb;
    hipStream_t s = R.main;
    if (alpha != T(1) && SB.mloc && nrhs_loc) slate_hip::gescale<K<T>>('G', SB.mloc, nrhs_loc, kv(alpha), kp(B), ldb, s);
    const bool lower = uplo == 'L';
    const i64 mloc_n = std::min(SA.mloc, numroc(n, nb, pr, p));
    for (i64 st = 0; st < nt; ++st) {
        const i64 k = lower ? nt - 1 - st : st;
        const i64 kb = std::min(nb, n - k * nb);
        const int rk = (int)(k % p), ck = (int)(k % q);
        const i64 lrk = tiles_before(k, p, pr) * nb, lck = tiles_before(k, q, pc) * nb;
        // this process row's rows of op(A)'s row k beyond the diagonal
        const i64 r0 = lower ? std::min(tiles_before(k + 1, p, pr) * nb, mloc_n) : 0;
        const i64 r1 = lower ? mloc_n : std::min(tiles_before(k, p, pr) * nb, mloc_n);
        const i64 nr = std::max<i64>(r1 - r0, 0);
        Scratch W((size_t)kb * std::max<i64>(nrhs_loc, 1) * sizeof(T), s);
        if (p > 1 || nr > 0) {
            Scratch Pn((size_t)std::max<i64>(nr, 1) * kb * sizeof(T), s);
            if (nr > 0) {
                if (pc == ck) copy2d(Pn.as<T>(), nr, A + r0 + lck * lda, lda, nr, kb, s);
                if (q > 1) gc->row->bcast(Pn.p, (size_t)nr * kb * sizeof(T), ck, s);
            }
            if (nrhs_loc) {
                if (nr > 0)
                    gemm_k<T>(tr, 'N', kb, nrhs_loc, nr, T(1), Pn.as<T>(), nr, B + r0, ldb, T(0), W.as<T>(), kb, s);
                else
                    slate_hip::geset<K<T>>('G', kb, nrhs_loc, kv(T(0)), kv(T(0)), kp(W.as<T>()), kb, s);
                if (p > 1) gc->col->allreduce(W.p, (size_t)kb * nrhs_loc, dt_of<T>::v, 's', s);
            }
        }
        if (pr == rk) {
            Scratch D((size_t)kb * kb * sizeof(T), s);
            if (pc == ck) copy2d(D.as<T>(), kb, A + lrk + lck * lda, lda, kb, kb, s);
            if (q > 1) gc->row->bcast(D.p, (size_t)kb * kb * sizeof(T), ck, s);
            if (nrhs_loc) {
                if (p > 1 || nr > 0)
                    slate_hip::geadd<K<T>>('G', kb, nrhs_loc, kv(T(-1)), kp(W.as<T>()), kb, kv(T(1)), kp(B + lrk), ldb,
                                           s);
                slate_hip::trsm<K<T>>('L', uplo, tr, diag, kb, nrhs_loc, kv(T(1)), kp(D.as<T>()), kb, kp(B + lrk),
                                      ldb, s);
            }
        }
    }
    NHIP(hipStreamSynchronize(s));
}

template <typename T>
void trsm(Side side, Uplo uplo, Op op, Diag diag, T alpha, const Matrix<T>& Av, Matrix<T>& B, const Options& opts) {
    NTRACE("trsm", nullptr);
    op = compose_op<T>(op, Av.op());
    const Matrix<T> A = Av.base();
    const Storage& SA = *A.storage();
    Storage& SB = *B.storage();
    const bool left = side == Side::Left;
    if (SA.m != SA.n || SA.n != (left ? SB.m : SB.n)) throw Error("native trsm: dimension mismatch");
    if (SA.nb != SB.nb || SA.p != SB.p || SA.q != SB.q) throw Error("native trsm: A and B must share grid and nb");
    NHIP(hipStreamSynchronize(rt().main));
    if (!left) {
        // X op(A) = alpha B  <=>  op(A)^T X^T = alpha B^T  (N, T), A X^H = conj(alpha) B^H (C):
        // a left solve on the transposed right-hand side
        const bool ch = op == Op::ConjTrans && is_cplx<T>();
        const Op bt = ch ? Op::ConjTrans : Op::Trans;
        Matrix<T> Y(SB.n, SB.m, SB.nb, SB.p, SB.q);
        copy<T>(bt, B, Y);
        const Op lop = op == Op::NoTrans ? Op::Trans : Op::NoTrans;
        trsm<T>(Side::Left, uplo, lop, diag, ch ? conj_of(alpha) : alpha, A, Y, opts);
        copy<T>(bt, Y, B);
        return;
    }
    if (op == Op::NoTrans) {
        trsm_left<T>((char)uplo, (char)diag, alpha, SA, SB);
        return;
    }
    trsm_left_t<T>((char)uplo, (char)diag, (op == Op::ConjTrans && is_cplx<T>()) ? 'C' : 'T', alpha, SA, SB);
}

template <typename T>
void copy(Op op, const Matrix<T>& Av, Matrix<T>& B) {
    op = compose_op<T>(op, Av.op());
    const Matrix<T> A = Av.base();
    const Storage& SA = *A.storage();
    Storage& SB = *B.storage();
    const bool tr = op != Op::NoTrans;
    if ((tr ? SA.n : SA.m) != SB.m || (tr ? SA.m : SA.n) != SB.n) throw Error("native copy: dimension mismatch");
    if (SA.nb != SB.nb || SA.p != SB.p || SA.q != SB.q) throw Error("native copy: A and B must share grid and nb");
    Runtime& R = rt();
    NHIP(hipStreamSynchronize(R.main));
    if (!tr) {
        copy2d(static_cast<T*>(SB.buf), SB.lld, static_cast<const T*>(SA.buf), SA.lld, SA.mloc, SA.nloc, R.main);
        NHIP(hipStreamSynchronize(R.main));
        return;
    }
    transpose_tiles<T>(SA, SB, (op == Op::ConjTrans && is_cplx<T>()) ? 'C' : 'T');
}

// tile (i, j) of L (m x n) -> tile (j, i) of U (n x m), transposed ('T') or
// conjugate-transposed ('C'), for every local tile of L: one batched
// point-to-point exchange (same-rank tiles are copied locally)
template <typename T>
static void transpose_tiles(const Storage& L, Storage& U, char ct) {
    Runtime& R = rt();
    hipStream_t s = R.main;
    const int p = L.p, q = L.q, pr = L.pr, pc = L.pc;
    const i64 nb = L.nb;
    const i64 mt = (L.m + nb - 1) / nb, ntl = (L.n + nb - 1) / nb;
    const T* A = static_cast<const T*>(L.buf);
    T* B = static_cast<T*>(U.buf);
    // tile t's extent: rows of L for i, columns of L for j
    auto mbr = [&](i64 t) { return std::min(nb, L.m - t * nb); };
    auto mbc = [&](i64 t) { return std::min(nb, L.n - t * nb); };
    auto owner = [&](i64 i, i64 j) { return (int)(i % p) + (int)(j % q) * p; };
    struct Item { i64 i, j; };
    std::map<int, std::vector<Item>> sends, recvs;
    for (i64 j = 0; j < ntl; ++j)
        for (i64 i = 0; i < mt; ++i) {
            const int src = owner(i, j), dst = owner(j, i);
            if (src == R.rank && dst == R.rank) {
                const T* a = A + tiles_before(i, p, pr) * nb + tiles_before(j, q, pc) * nb * L.lld;
                T* b = B + tiles_before(j, p, pr) * nb + tiles_before(i, q, pc) * nb * U.lld;
                slate_hip::gecopy<K<T>, K<T>>('G', ct, mbc(j), mbr(i), kp(a), L.lld, kp(b), U.lld, s);
            } else if (src == R.rank) {
                sends[dst].push_back({i, j});
            } else if (dst == R.rank) {
                recvs[src].push_back({i, j});
            }
        }
    std::vector<std::unique_ptr<Scratch>> bufs;
    std::vector<P2P> ops;
    std::vector<std::tuple<Scratch*, std::vector<Item>*>> unpack;
    for (auto& kv2 : sends) {
        size_t tot = 0;
        for (auto& it : kv2.second) tot += (size_t)mbr(it.i) * mbc(it.j);
        bufs.push_back(std::make_unique<Scratch>(tot * sizeof(T), s));
        size_t off = 0;
        for (auto& it : kv2.second) {
            const T* a = A + tiles_before(it.i, p, pr) * nb + tiles_before(it.j, q, pc) * nb * L.lld;
            copy2d(bufs.back()->as<T>() + off, mbr(it.i), a, L.lld, mbr(it.i), mbc(it.j), s);
            off += (size_t)mbr(it.i) * mbc(it.j);
        }
        ops.push_back({true, kv2.first, bufs.back()->p, tot * sizeof(T)});
    }
    for (auto& kv2 : recvs) {
        size_t tot = 0;
        for (auto& it : kv2.second) tot += (size_t)mbr(it.i) * mbc(it.j);
        bufs.push_back(std::make_unique<Scratch>(tot * sizeof(T), s));
        ops.push_back({false, kv2.first, bufs.back()->p, tot * sizeof(T)});
        unpack.emplace_back(bufs.back().get(), &kv2.second);
    }
    if (!ops.empty()) world_comm()->exchange(ops, s);
    for (auto& u : unpack) {
        Scratch* b = std::get<0>(u);
        size_t off = 0;
        for (auto& it : *std::get<1>(u)) {
            T* dst = B + tiles_before(it.j, p, pr) * nb + tiles_before(it.i, q, pc) * nb * U.lld;
            slate_hip::gecopy<K<T>, K<T>>('G', ct, mbc(it.j), mbr(it.i), kp(b->as<T>() + off), mbr(it.i), kp(dst), U.lld,
                                          s);
            off += (size_t)mbr(it.i) * mbc(it.j);
        }
    }
    NHIP(hipStreamSynchronize(s));
}

// ------------------------------------------------------------ solves
template <typename T>
int64_t potrs(const HermitianMatrix<T>& A, Matrix<T>& B, const Options& opts) {
    trsm<T>(Side::Left, Uplo::Lower, Op::NoTrans, Diag::NonUnit, T(1), A, B, opts);
    trsm<T>(Side::Left, Uplo::Lower, Op::ConjTrans, Diag::NonUnit, T(1), A, B, opts);
    return 0;
}

template <typename T>
int64_t posv(HermitianMatrix<T>& A, Matrix<T>& B, const Options& opts) {
    const int64_t info = potrf(A, opts);
    if (info == 0) potrs(A, B, opts);
    return info;
}

// ------------------------------------------------------------ getrf
// row interchanges ipiv[k1, k2) (global rows, 0-based, sequential) applied to
// the local columns [c0, c1) of a p x q matrix: p == 1 a local laswp; p > 1
// the owner-masked exchange (swap plan folded on the device, pack the rows
// this rank owns, all-reduce over the process column, unpack) in chunks of
// at most 512 swaps -- models/lu.py permute_rows / _xchg_update
template <typename T>
static void permute_rows_dist(Storage& S, const i64* ipiv_d, i64 k1, i64 k2, i64 c0, i64 c1, int incx, hipStream_t s,
                              Comm* colc) {
    if (c1 <= c0 || k2 <= k1) return;
    T* buf = static_cast<T*>(S.buf);
    if (S.p == 1) {
        slate_hip::laswp_off<K<T>>(c1 - c0, kp(buf + c0 * S.lld), S.lld, k1, k2, ipiv_d, 0, s, incx);
        return;
    }
    Scratch plan(slate_hip::swap_plan_bytes(), s);
    std::vector<std::pair<i64, i64>> ch;
    for (i64 a = k1; a < k2; a += 512) ch.push_back({a, std::min(k2, a + 512)});
    if (incx < 0) std::reverse(ch.begin(), ch.end());
    for (auto& c : ch) {
        const i64 ns = c.second - c.first, S2 = 2 * ns;
        slate_hip::swap_plan(c.first, c.second, ipiv_d, 0, incx, plan.p, s);
        Scratch X((size_t)S2 * (c1 - c0) * sizeof(T), s);
        slate_hip::xchg_gather<K<T>>(plan.p, S2, c1 - c0, kp(buf + c0 * S.lld), S.lld, kp(X.as<T>()), S2, S.nb, S.p,
                                     S.pr, s);
        colc->allreduce(X.p, (size_t)S2 * (c1 - c0), dt_of<T>::v, 's', s);
        slate_hip::xchg_scatter<K<T>>(plan.p, S2, c1 - c0, kp(X.as<T>()), S2, kp(buf + c0 * S.lld), S.lld, S.nb, S.p,
                                      S.pr, s);
    }
}

// Exact row moves of one LU step for p > 1 (models/lu.py _p2p_rows /
// internal::permuteRows): the step's swap sequence folded on the host into
// (destination, source) global rows; rows staying inside this process row
// move locally, rows changing process row travel point-to-point (one
// batched exchange on the column communicator, rows in destination order
// on both sides) -- only the rows that change owner move, over every local
// column range at once.  g_lu_xchg counts the bytes this rank sent.
static std::vector<std::pair<i64, i64>> fold_moves(const std::vector<i64>& pv, i64 r0) {
    std::map<i64, i64> cur;                  // position -> original row now there
    for (size_t i = 0; i < pv.size(); ++i) {
        const i64 a = r0 + (i64)i, b = r0 + pv[i];
        if (a == b) continue;
        const i64 ca = cur.count(a) ? cur[a] : a, cb = cur.count(b) ? cur[b] : b;
        cur[a] = cb;
        cur[b] = ca;
    }
    std::vector<std::pair<i64, i64>> mv;
    for (auto& x : cur)
        if (x.first != x.second) mv.push_back(x);
    return mv;                               // sorted by destination
}

static std::atomic<long long> g_lu_xchg_bytes{0}, g_lu_xchg_rows{0};

template <typename T>
static void p2p_rows(Storage& S, const std::vector<std::pair<i64, i64>>& mv,
                     const std::vector<std::pair<i64, i64>>& ranges, Comm* colc, hipStream_t s) {
    i64 W = 0;
    for (auto& r : ranges) W += std::max<i64>(r.second - r.first, 0);
    if (W == 0 || mv.empty()) return;
    const i64 nb = S.nb;
    const int p = S.p, pr = S.pr;
    auto own = [&](i64 g) { return (int)((g / nb) % p); };
    auto loc = [&](i64 g) { return (g / (nb * p)) * nb + g % nb; };
    std::map<int, std::vector<i64>> sends, recvs;
    std::vector<i64> ld, ls;
    long long cross = 0;
    for (auto& x : mv) {
        const int od = own(x.first), os = own(x.second);
        cross += od != os;
        if (os == pr && od != pr) sends[od].push_back(loc(x.second));
        else if (od == pr && os != pr) recvs[os].push_back(loc(x.first));
        else if (od == pr && os == pr) { ld.push_back(loc(x.first)); ls.push_back(loc(x.second)); }
    }
    // every index list in one upload: [sends per peer | recvs per peer | ls | ld]
    std::vector<i64> flat;
    std::vector<std::pair<int, size_t>> soff, roff;
    for (auto& kv2 : sends) { soff.push_back({kv2.first, flat.size()}); flat.insert(flat.end(), kv2.second.begin(), kv2.second.end()); }
    for (auto& kv2 : recvs) { roff.push_back({kv2.first, flat.size()}); flat.insert(flat.end(), kv2.second.begin(), kv2.second.end()); }
    const size_t lso = flat.size();
    flat.insert(flat.end(), ls.begin(), ls.end());
    const size_t ldo = flat.size();
    flat.insert(flat.end(), ld.begin(), ld.end());
    if (flat.empty()) return;
    Scratch idx(flat.size() * sizeof(i64), s);
    upload(idx.p, flat.data(), flat.size() * sizeof(i64), s);
    const i64* id = idx.as<i64>();
    T* buf = static_cast<T*>(S.buf);
    // gather c rows (local indices at id + o) of every range into X (c x W)
    auto gather = [&](T* X, i64 c, size_t o) {
        i64 off = 0;
        for (auto& r : ranges) {
            const i64 w = r.second - r.first;
            if (w <= 0) continue;
            slate_hip::permute_rows_gather<K<T>>(c, w, kp(buf + r.first * S.lld), S.lld, kp(X + off * c), c, id + o, s);
            off += w;
        }
    };
    auto scatter = [&](const T* X, i64 c, size_t o) {
        i64 off = 0;
        for (auto& r : ranges) {
            const i64 w = r.second - r.first;
            if (w <= 0) continue;
            slate_hip::permute_rows_scatter<K<T>>(c, w, kp(X + off * c), c, kp(buf + r.first * S.lld), S.lld, id + o, s);
            off += w;
        }
    };
    std::vector<std::unique_ptr<Scratch>> bufs;
    std::vector<P2P> ops;
    std::vector<std::tuple<Scratch*, i64, size_t>> unpack;
    long long sent = 0;
    for (auto& so : soff) {
        const i64 c = (i64)sends[so.first].size();
        bufs.push_back(std::make_unique<Scratch>((size_t)c * W * sizeof(T), s));
        gather(bufs.back()->as<T>(), c, so.second);
        ops.push_back({true, so.first, bufs.back()->p, (size_t)c * W * sizeof(T)});
        sent += (long long)c * W * sizeof(T);
    }
    for (auto& ro : roff) {
        const i64 c = (i64)recvs[ro.first].size();
        bufs.push_back(std::make_unique<Scratch>((size_t)c * W * sizeof(T), s));
        ops.push_back({false, ro.first, bufs.back()->p, (size_t)c * W * sizeof(T)});
        unpack.emplace_back(bufs.back().get(), c, ro.second);
    }
    const i64 nl = (i64)ls.size();
    std::unique_ptr<Scratch> tmp;
    if (nl) {                                // all local sources read before any is overwritten
        tmp = std::make_unique<Scratch>((size_t)nl * W * sizeof(T), s);
        gather(tmp->as<T>(), nl, lso);
    }
    if (!ops.empty()) colc->exchange(ops, s);
    for (auto& u : unpack) scatter(std::get<0>(u)->as<T>(), std::get<1>(u), std::get<2>(u));
    if (nl) scatter(tmp->as<T>(), nl, ldo);
    g_lu_xchg_bytes += sent;
    g_lu_xchg_rows += cross;
}

// LU of the p x q panel column k (kb columns at local column lck of the
// process column that owns it): rows stay on their owners, one record
// all-gather per column (lu_dist_step), recursion halves joined by the
// owner-masked row exchange; every rank of the column ends with its factored
// rows in place and the same kb x kb top block T
template <typename T>
static void panel_dist(Storage& S, i64 k, i64 kb, i64 lck, i64* ipiv_d, i64* info, double thr, int bw, T* Tt,
                       const i64* grow_d, hipStream_t s) {
    const int p = S.p, pr = S.pr;
    const i64 nb = S.nb, r0 = k * nb;
    const int rk = (int)(k % p);
    const i64 lr_k = std::min(tiles_before(k, p, pr) * nb, S.mloc);
    const i64 nmine = S.mloc - lr_k;
    T* buf = static_cast<T*>(S.buf);
    T* W = buf + lr_k + lck * S.lld;
    const i64 ldw = S.lld;
    Comm* colc = S.gc->col.get();
    Scratch part(2 * 1024 * 8 + 64, s);
    const int b = std::max(1, bw);
    Scratch recs((size_t)p * (3 + 2 * b) * sizeof(T), s), rec((size_t)(3 + 2 * b) * sizeof(T), s);
    dzero(Tt, (size_t)kb * kb * sizeof(T), s);
    i64* piv = ipiv_d + r0;                 // panel-relative
    PeerBox* pbx = b <= slate_hip::lu_peer_max_b() ? peer_box(colc, S.gc->colpeer, s) : nullptr;
    auto base = [&](i64 c0, i64 c1) {
        if (pbx) {
            // ONE persistent launch per block; the column peers trade their
            // records through the peer-mapped mailboxes (no host round trip)
            slate_hip::LuPeer pe{pbx->mbox_d, p, colc->rank, pbx->part, pbx->seq, pr == rk ? 1 : 0, pbx->err};
            pbx->seq += (c1 - c0) + 1;
            ++pbx->launches;
            const int G = (int)std::max<i64>(1, std::min<i64>(64, (nmine + 1023) / 1024));
            slate_hip::lu_dist_base<K<T>>(nmine, kp(nmine ? W + c0 * ldw : buf), ldw, grow_d, (int)c0, (int)c1, kp(Tt),
                                          kb, piv, info, 0, thr, pe, G, s);
            return;
        }
        const int recn = 3 + 2 * (int)(c1 - c0);
        for (i64 j = c0; j <= c1; ++j) {
            const bool nxt = j < c1;
            const i64 dl = (pr == rk && nxt) ? j : -1;
            slate_hip::lu_dist_step<K<T>>(nmine, kp(W + c0 * ldw), ldw, grow_d, (int)c0, (int)c1, (int)j,
                                          j > c0 ? kp(recs.as<T>()) : nullptr, p, kp(Tt), kb, piv, info, 0, thr,
                                          kp(rec.as<T>()), part.p, dl, s);
            if (nxt) colc->allgather(rec.p, recs.p, (size_t)recn * sizeof(T), s);
        }
    };
    // interchanges of panel columns [a, e) applied to panel columns [ca, cb);
    // returns the window rows (new rows a..e) in a buffer of e - a rows
    auto exchange = [&](i64 a, i64 e, i64 ca, i64 cb, std::unique_ptr<Scratch>& Xout) -> T* {
        Scratch plan(slate_hip::swap_plan_bytes(), s);
        slate_hip::swap_plan(r0 + a, r0 + e, ipiv_d, -r0, 1, plan.p, s);
        const i64 S2 = 2 * (e - a), w = cb - ca;
        Xout = std::make_unique<Scratch>((size_t)S2 * w * sizeof(T), s);
        T* X = Xout->as<T>();
        T* cols = buf + (lck + ca) * S.lld;
        slate_hip::xchg_gather<K<T>>(plan.p, S2, w, kp(cols), S.lld, kp(X), S2, nb, p, pr, s);
        colc->allreduce(X, (size_t)S2 * w, dt_of<T>::v, 's', s);
        slate_hip::xchg_scatter<K<T>>(plan.p, S2, w, kp(X), S2, kp(cols), S.lld, nb, p, pr, s);
        return X;                           // leading dimension S2
    };
    std::function<void(i64, i64)> rec_fn = [&](i64 c0, i64 c1) {
        if (c1 - c0 <= b) { base(c0, c1); return; }
        i64 cm = c0 + ((c1 - c0) / 2 + b - 1) / b * b;
        if (cm >= c1) cm = c1 - b;
        rec_fn(c0, cm);
        std::unique_ptr<Scratch> Xs;
        T* U = exchange(c0, cm, cm, c1, Xs);
        const i64 ldu = 2 * (cm - c0);
        slate_hip::trsm<K<T>>('L', 'L', 'N', 'U', cm - c0, c1 - cm, kv(T(1)), kp(Tt + c0 + c0 * kb), kb, kp(U), ldu, s);
        copy2d(Tt + c0 + cm * kb, kb, U, ldu, cm - c0, c1 - cm, s);
        if (pr == rk) copy2d(W + c0 + cm * ldw, ldw, U, ldu, cm - c0, c1 - cm, s);
        const i64 i0 = pr == rk ? cm : 0;
        if (nmine > i0)
            gemm_k<T>('N', 'N', nmine - i0, c1 - cm, cm - c0, T(-1), W + i0 + c0 * ldw, ldw, U, ldu, T(1),
                      W + i0 + cm * ldw, ldw, s);
        rec_fn(cm, c1);
        std::unique_ptr<Scratch> X2;
        T* V = exchange(cm, c1, c0, cm, X2);
        copy2d(Tt + cm + c0 * kb, kb, V, 2 * (c1 - cm), c1 - cm, cm - c0, s);
    };
    rec_fn(0, kb);
}

// bytes this rank sent and rows that changed process row in the exact LU
// row exchanges since the last call (tests, examples)
void lu_exchange_stats(long long* bytes, long long* rows) {
    if (bytes) *bytes = g_lu_xchg_bytes.exchange(0);
    if (rows) *rows = g_lu_xchg_rows.exchange(0);
}

// ------------------------------------------------------------ CALU (tournament pivoting)
// Reference: src/getrf_tntpiv.cc, src/internal/internal_getrf_tntpiv.cc
// (Grigori, Demmel, Xiang).  The play-offs are the persistent partial-
// pivoting LU panel on row blocks; the winners' ORIGINAL rows meet in the
// next round (device row gathers), the winners of the last round, in its
// pivot order, become the panel's LAPACK-style interchanges.

// one play-off: partial-pivoting LU of a copy of the R x w rows A (ld lda);
// the min(R, kb) winners (row indices into A) in pivot order; with keep the
// factored copy (ld R, rows permuted) stays in *keep
template <typename T>
static std::vector<i64> calu_playoff(i64 R, i64 w, i64 kb, const T* A, i64 lda, double thr, i64* info_d,
                                     std::unique_ptr<Scratch>* keep, hipStream_t s) {
    const i64 c = std::min(R, kb);
    auto W = std::make_unique<Scratch>(sizeof(T) * std::max<i64>(R, 1) * w, s);
    copy2d(W->as<T>(), R, A, lda, R, w, s);
    Scratch lp(sizeof(i64) * std::max<i64>(c, 1), s);
    dzero(lp.p, sizeof(i64) * std::max<i64>(c, 1), s);
    slate_hip::getrf_panel_ws<K<T>>(R, std::min(w, kb), kp(W->as<T>()), R, lp.as<i64>(), info_d, thr, false,
                                    rt().lu_work, s);
    std::vector<i64> h((size_t)std::max<i64>(c, 1));
    NHIP(hipMemcpyAsync(h.data(), lp.p, sizeof(i64) * h.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    std::vector<i64> idx((size_t)R);
    for (i64 i = 0; i < R; ++i) idx[i] = i;
    for (i64 i = 0; i < c; ++i) std::swap(idx[i], idx[h[i]]);
    idx.resize((size_t)c);
    if (keep) *keep = std::move(W);
    return idx;
}

// rows sel (into A, ld lda) gathered into a new |sel| x w block
template <typename T>
static std::unique_ptr<Scratch> calu_gather(const std::vector<i64>& sel, i64 w, const T* A, i64 lda, hipStream_t s) {
    const i64 r = (i64)sel.size();
    auto C = std::make_unique<Scratch>(sizeof(T) * std::max<i64>(r, 1) * w, s);
    Scratch pd(sizeof(i64) * std::max<i64>(r, 1), s);
    upload(pd.p, sel.data(), sizeof(i64) * r, s);
    slate_hip::permute_rows_gather<K<T>>(r, w, kp(A), lda, kp(C->as<T>()), r, pd.as<i64>(), s);
    NHIP(hipStreamSynchronize(s));
    return C;
}

// local tournament over the R rows of A: at most kb nominees (indices into
// A); every round plays blocks of `leaf` (>= 2 kb) rows
template <typename T>
static std::vector<i64> calu_local(i64 R, i64 w, i64 kb, const T* A, i64 lda, double thr, i64 leaf, i64* info_d,
                                   hipStream_t s) {
    std::vector<i64> cand;
    for (i64 a = 0; a < R; a += leaf) {
        const i64 r = std::min(leaf, R - a);
        for (i64 i : calu_playoff<T>(r, w, kb, A + a, lda, thr, info_d, nullptr, s)) cand.push_back(a + i);
    }
    while ((i64)cand.size() > kb) {
        std::vector<i64> next;
        for (size_t g = 0; g < cand.size(); g += (size_t)leaf) {
            const size_t e = std::min(cand.size(), g + (size_t)leaf);
            std::vector<i64> grp(cand.begin() + g, cand.begin() + e);
            auto C = calu_gather<T>(grp, w, A, lda, s);
            for (i64 i : calu_playoff<T>((i64)grp.size(), w, kb, C->template as<T>(), (i64)grp.size(), thr, info_d, nullptr, s))
                next.push_back(grp[i]);
        }
        cand.swap(next);
    }
    return cand;
}

// selected rows (pivot order, panel-relative) -> LAPACK sequential interchanges
static std::vector<i64> calu_ipiv(const std::vector<i64>& sel, i64 mk) {
    std::vector<i64> at((size_t)mk), pos((size_t)mk), piv(sel.size());
    for (i64 i = 0; i < mk; ++i) at[i] = pos[i] = i;
    for (size_t i = 0; i < sel.size(); ++i) {
        const i64 p = pos[sel[i]];
        piv[i] = p;
        const i64 ri = at[i], rp = at[p];
        std::swap(at[i], at[p]);
        pos[ri] = p;
        pos[rp] = (i64)i;
    }
    return piv;
}

// 1 x q: the panel (mk x wk at A) on one rank
template <typename T>
static void calu_panel_1(i64 mk, i64 wk, T* A, i64 lda, i64* piv_d, i64* info, double thr, i64 leaf, hipStream_t s) {
    const i64 kb = std::min(mk, wk);
    Scratch dinfo(sizeof(i64), s);
    dzero(dinfo.p, sizeof(i64), s);
    std::vector<i64> sel = calu_local<T>(mk, wk, kb, A, lda, thr, std::max<i64>(leaf, 2 * kb), dinfo.as<i64>(), s);
    if ((i64)sel.size() > kb) sel.resize((size_t)kb);
    const std::vector<i64> piv = calu_ipiv(sel, mk);
    upload(piv_d, piv.data(), sizeof(i64) * piv.size(), s);
    slate_hip::laswp_off<K<T>>(wk, kp(A), lda, 0, (i64)piv.size(), piv_d, 0, s);
    Scratch np(sizeof(i64) * std::max<i64>(kb, 1), s);
    slate_hip::getrf_panel_ws<K<T>>(mk, wk, kp(A), lda, np.as<i64>(), info, thr, true, rt().lu_work, s);
}

// p > 1: local play-offs on every rank of the panel's process column, ONE
// all-gather of the (<= kb) nominees per rank, the final round redundantly
// on the column; then the exact row exchange of the panel columns, U11 / L11
// from the final round, L21 = A21 U11^-1 (same outputs as panel_dist)
template <typename T>
static void calu_panel_dist(Storage& S, i64 k, i64 kb, i64 lck, i64* ipiv_d, i64* info, double thr, i64 leaf, T* Tt,
                            hipStream_t s) {
    const int p = S.p, pr = S.pr;
    const i64 nb = S.nb, r0 = k * nb;
    const int rk = (int)(k % p);
    const i64 lr_k = std::min(tiles_before(k, p, pr) * nb, S.mloc);
    const i64 nmine = S.mloc - lr_k;
    T* buf = static_cast<T*>(S.buf);
    T* W = buf + lr_k + lck * S.lld;
    Comm* colc = S.gc->col.get();
    Scratch dinfo(sizeof(i64), s);
    dzero(dinfo.p, sizeof(i64), s);
    std::vector<i64> loc;
    if (nmine) loc = calu_local<T>(nmine, kb, kb, W, S.lld, thr, std::max<i64>(leaf, 2 * kb), dinfo.as<i64>(), s);
    // pack: kb x kb nominee rows (ld kb) + kb panel-relative global row ids (-1: none)
    const size_t rb = sizeof(T) * kb * kb, ib = sizeof(i64) * kb, pkb = rb + ib;
    Scratch pk(pkb, s), all(pkb * p, s);
    dzero(pk.p, pkb, s);
    std::vector<i64> gid((size_t)kb, -1);
    for (size_t i = 0; i < loc.size(); ++i) gid[i] = l2g(lr_k + loc[i], nb, p, pr) - r0;
    if (!loc.empty()) {
        auto C = calu_gather<T>(loc, kb, W, S.lld, s);
        copy2d(pk.as<T>(), kb, C->template as<T>(), (i64)loc.size(), (i64)loc.size(), kb, s);
    }
    upload(static_cast<char*>(pk.p) + rb, gid.data(), ib, s);
    colc->allgather(pk.p, all.p, pkb, s);
    std::vector<i64> gall((size_t)kb * p);
    for (int r = 0; r < p; ++r)
        NHIP(hipMemcpyAsync(gall.data() + (size_t)r * kb, static_cast<char*>(all.p) + pkb * r + rb, ib,
                            hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    // the stack of every rank's nominees, in rank order
    std::vector<i64> sg;
    i64 tot = 0;
    for (int r = 0; r < p; ++r)
        for (i64 i = 0; i < kb; ++i)
            if (gall[(size_t)r * kb + i] >= 0) ++tot;
    Scratch stk(sizeof(T) * std::max<i64>(tot, 1) * kb, s);
    i64 o = 0;
    for (int r = 0; r < p; ++r) {
        i64 c = 0;
        while (c < kb && gall[(size_t)r * kb + c] >= 0) ++c;
        copy2d(stk.as<T>() + o, tot, reinterpret_cast<T*>(static_cast<char*>(all.p) + pkb * r), kb, c, kb, s);
        for (i64 i = 0; i < c; ++i) sg.push_back(gall[(size_t)r * kb + i]);
        o += c;
    }
    std::unique_ptr<Scratch> F;
    const std::vector<i64> win = calu_playoff<T>(tot, kb, kb, stk.as<T>(), tot, thr, info, &F, s);
    std::vector<i64> sel;
    for (i64 i : win) sel.push_back(sg[i]);
    const std::vector<i64> piv = calu_ipiv(sel, S.m - r0);
    upload(ipiv_d + r0, piv.data(), sizeof(i64) * piv.size(), s);
    // LU11 (the final round's top kb rows) -> Tt
    copy2d(Tt, kb, F->as<T>(), tot, kb, kb, s);
    // the winners into the panel's top rows (owner-masked all-reduce exchange)
    Scratch plan(slate_hip::swap_plan_bytes(), s);
    slate_hip::swap_plan(r0, r0 + kb, ipiv_d, -r0, 1, plan.p, s);
    const i64 S2 = 2 * kb;
    Scratch X((size_t)S2 * kb * sizeof(T), s);
    T* cols = buf + lck * S.lld;
    slate_hip::xchg_gather<K<T>>(plan.p, S2, kb, kp(cols), S.lld, kp(X.as<T>()), S2, nb, p, pr, s);
    colc->allreduce(X.p, (size_t)S2 * kb, dt_of<T>::v, 's', s);
    slate_hip::xchg_scatter<K<T>>(plan.p, S2, kb, kp(X.as<T>()), S2, kp(cols), S.lld, nb, p, pr, s);
    if (pr == rk) copy2d(W, S.lld, Tt, kb, kb, kb, s);
    const i64 i0 = pr == rk ? kb : 0;
    if (nmine > i0)
        slate_hip::trsm<K<T>>('R', 'U', 'N', 'N', nmine - i0, kb, kv(T(1)), kp(Tt), kb, kp(W + i0), S.lld, s);
}

template <typename T>
int64_t getrf_tntpiv(Matrix<T>& A, std::vector<int64_t>& ipiv, const Options& opts) {
    Options o = opts;
    o.lu_method = 1;
    return getrf<T>(A, ipiv, o);
}

// 1 x q LU with RowMajor rows (SLATE getrf.cc:51-55 on GPUs; models/lu.py
// _getrf_p1 with T): the local block is factored TRANSPOSED, T = buf^T
// (nloc x m, ld ldt), so a row interchange of A swaps two contiguous columns
// of T (whole cache lines, one folded swap plan per step for every column
// range) and the trailing update is the NT GEMM T22 -= U12^T L21^T.  Each
// panel is copied out column-major into a ring slot for the persistent
// panel kernel and written back transposed.  Wide trailing ranges take the
// U rows from the explicit L11 inverse (one GEMM instead of the blocked
// substitution); buf stays intact until the final copy back, so a step
// whose inverse grew beyond SLATE_AMD_LU_INV_GROWTH (1e6) makes the caller
// redo the factorization with the substitution (returns true).
template <typename T>
static bool getrf_p1_rm(Storage& S, int la, double thr, i64* ipiv_d, i64* infos, bool no_inv) {
    using Rl = real_t<T>;
    Runtime& R = rt();
    GridComms* gc = S.gc;
    const int q = S.q, pc = S.pc;
    const i64 nb = S.nb, m = S.m, n = S.n, lld = S.lld, nloc = S.nloc;
    const i64 kt = std::min((m + nb - 1) / nb, (n + nb - 1) / nb);
    T* buf = static_cast<T*>(S.buf);
    hipStream_t ps = R.panel, us = R.update;
    const i64 ldt = std::max<i64>(1, (nloc + 7) / 8 * 8);
    Scratch Tm((size_t)ldt * std::max<i64>(m, 1) * sizeof(T), R.main);
    T* Tt = Tm.as<T>();
    const i64 inv_min = no_inv ? 0 : env_int("SLATE_AMD_LU_INV_MIN", 4096);
    Scratch growth(sizeof(Rl) * (size_t)std::max<i64>(kt, 1), R.main);
    dzero(growth.p, sizeof(Rl) * (size_t)std::max<i64>(kt, 1), R.main);
    join(R.main, ps);
    join(R.main, us);
    const int NR = la + 3;
    std::vector<std::unique_ptr<Scratch>> ring;
    for (int r = 0; r < NR; ++r) ring.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(m, 1) * nb * sizeof(T), ps));
    std::vector<std::unique_ptr<Scratch>> plans((size_t)kt), linv((size_t)kt);
    std::vector<std::unique_ptr<Event>> ev_tr((size_t)kt), ev_used((size_t)kt);
    std::vector<std::array<i64, 2>> left;            // (step, left columns)
    const i64 tail = (i64)(kt * 0.6);
    // buf -> T: the bulk on the update stream, concurrently with panel 0
    // (which reads buf itself); the lookahead columns on the panel stream
    const i64 lcla0 = std::min(tiles_before(1 + la, q, pc) * nb, nloc);
    if (nloc > lcla0 && m > 0)
        slate_hip::gecopy<K<T>, K<T>>('G', 'T', nloc - lcla0, m, kp(buf + lcla0 * lld), lld, kp(Tt + lcla0), ldt, us);
    for (i64 k = 0; k < kt; ++k) {
        const i64 r0 = k * nb;
        const i64 kb = std::min({nb, n - r0, m - r0});
        const i64 mk = m - r0;
        const bool own = (k % q) == pc;
        const i64 lck = tiles_before(k, q, pc) * nb;
        const i64 lc1 = std::min(tiles_before(k + 1, q, pc) * nb, nloc);
        const i64 lcla = std::min(tiles_before(k + 1 + la, q, pc) * nb, nloc);
        if (k - la - 1 >= 0) ev_tr[k - la - 1]->wait(ps);
        if (k >= NR) ev_used[k - NR]->wait(ps);
        T* Lp = ring[k % NR]->as<T>();
        const i64 ldl = mk;
        {
            NTRACE("getrf::panel", ps);
            if (own) {
                const i64 wk = std::min(nb, n - r0);
                if (k == 0) copy2d(Lp, ldl, buf + r0 + lck * lld, lld, mk, wk, ps);
                else slate_hip::gecopy<K<T>, K<T>>('G', 'T', mk, wk, kp(Tt + lck + r0 * ldt), ldt, kp(Lp), ldl, ps);
                slate_hip::getrf_panel_ws<K<T>>(mk, wk, kp(Lp), ldl, ipiv_d + r0, infos + k, thr, false, R.lu_work, ps);
                slate_hip::gecopy<K<T>, K<T>>('G', 'T', wk, mk, kp(Lp), ldl, kp(Tt + lck + r0 * ldt), ldt, ps);
            }
            if (q > 1) {
                gc->row->bcast(ipiv_d + r0, (size_t)kb * sizeof(i64), (int)(k % q), ps);
                gc->row->bcast(Lp, (size_t)mk * kb * sizeof(T), (int)(k % q), ps);
            }
            plans[k] = std::make_unique<Scratch>(slate_hip::swap_plan_bytes(), ps);
            slate_hip::swap_plan(r0, r0 + kb, ipiv_d, -r0, 1, plans[k]->p, ps);
        }
        const T* Li = nullptr;
        if (inv_min && nloc - lcla >= inv_min && kb == nb) {
            linv[k] = std::make_unique<Scratch>((size_t)kb * kb * sizeof(T), ps);
            slate_hip::tri_inv<K<T>>('L', 'U', kb, kp(Lp), ldl, kp(linv[k]->template as<T>()), kb, ps);
            Scratch cm((size_t)(2 * kb + 2) * sizeof(Rl), ps), c1v((size_t)(kb + 2) * sizeof(Rl), ps);
            slate_hip::genorm<K<T>, Rl>('M', 'G', 'N', 0, kb, kb, kp(linv[k]->template as<T>()), kb, cm.as<Rl>(), ps);
            slate_hip::genorm<Rl, Rl>('M', 'G', 'N', 0, kb, 1, cm.as<Rl>(), kb, c1v.as<Rl>(), ps);
            dcopy(growth.as<Rl>() + k, c1v.p, sizeof(Rl), ps);
            Li = linv[k]->template as<T>();
        }
        const void* plan = plans[k]->p;
        auto update = [&](i64 c0, i64 c1, hipStream_t s) {
            if (c1 <= c0) return;
            const i64 w = c1 - c0;
            slate_hip::laswp_cols_plan<K<T>>(w, kp(Tt + c0), ldt, plan, s);
            T* Ut = Tt + c0 + r0 * ldt;
            if (Li) {
                Scratch tmp((size_t)w * kb * sizeof(T), s);
                copy2d(tmp.as<T>(), w, Ut, ldt, w, kb, s);
                gemm_k<T>('N', 'T', w, kb, kb, T(1), tmp.as<T>(), w, Li, kb, T(0), Ut, ldt, s);
            } else {
                slate_hip::trsm<K<T>>('R', 'L', 'T', 'U', w, kb, kv(T(1)), kp(Lp), ldl, kp(Ut), ldt, s);
            }
            if (m > r0 + kb)
                gemm_k<T>('N', 'T', w, m - r0 - kb, kb, T(-1), Ut, ldt, Lp + kb, ldl, T(1), Tt + c0 + (r0 + kb) * ldt,
                          ldt, s);
        };
        if (k >= 1 && la > 0) ev_tr[k - 1]->wait(ps);
        if (k == 0 && lcla > lc1)
            slate_hip::gecopy<K<T>, K<T>>('G', 'T', lcla - lc1, m, kp(buf + lc1 * lld), lld, kp(Tt + lc1), ldt, ps);
        {
            NTRACE("getrf::lookahead", ps);
            update(lc1, lcla, ps);
        }
        Event ev_panel;
        ev_panel.record(ps);
        ev_panel.wait(us);
        const i64 lcnx = std::max(std::min(tiles_before(k + 2 + la, q, pc) * nb, nloc), lcla);
        {
            NTRACE("getrf::update", us);
            update(lcla, lcnx, us);
            ev_tr[k] = std::make_unique<Event>();
            ev_tr[k]->record(us);
            update(lcnx, nloc, us);
        }
        // the factored columns left of the panel: their interchanges are
        // deferred into the panel-bound tail and spread over its steps
        if (lck > 0) left.push_back({k, lck});
        if (k >= tail) {
            const i64 todo = ((i64)left.size() + std::max<i64>(1, kt - k) - 1) / std::max<i64>(1, kt - k);
            for (i64 t = 0; t < todo && !left.empty(); ++t) {
                const auto it = left.front();
                left.erase(left.begin());
                slate_hip::laswp_cols_plan<K<T>>(it[1], kp(Tt), ldt, plans[it[0]]->p, us);
            }
        }
        ev_used[k] = std::make_unique<Event>();
        ev_used[k]->record(us);
    }
    for (auto& it : left) slate_hip::laswp_cols_plan<K<T>>(it[1], kp(Tt), ldt, plans[it[0]]->p, us);
    join(us, ps);
    join(ps, R.main);
    for (auto& x : ring) x->s = R.main;
    for (auto& x : plans) if (x) x->s = R.main;
    for (auto& x : linv) if (x) x->s = R.main;
    if (inv_min) {
        const double lim = [] { const char* e = std::getenv("SLATE_AMD_LU_INV_GROWTH"); return e ? std::atof(e) : 1e6; }();
        std::vector<Rl> g((size_t)std::max<i64>(kt, 1));
        NHIP(hipMemcpyAsync(g.data(), growth.p, g.size() * sizeof(Rl), hipMemcpyDeviceToHost, R.main));
        NHIP(hipStreamSynchronize(R.main));
        for (Rl v : g)
            if (!((double)v <= lim)) return true;       // NaN or too large: redo with the substitution
    }
    if (nloc && m) slate_hip::gecopy<K<T>, K<T>>('G', 'T', m, nloc, kp(Tt), ldt, kp(buf), lld, R.main);
    NHIP(hipStreamSynchronize(R.main));
    return false;
}

template <typename T>
int64_t getrf(Matrix<T>& A, std::vector<int64_t>& ipiv_out, const Options& opts) {
    NTRACE("getrf", nullptr);
    Storage& S = *A.storage();
    Runtime& R = rt();
    GridComms* gc = S.gc;
    const int p = S.p, q = S.q, pr = S.pr, pc = S.pc;
    const i64 nb = S.nb, m = S.m, n = S.n, lld = S.lld, nloc = S.nloc, mloc = S.mloc;
    const i64 kt = std::min((m + nb - 1) / nb, (n + nb - 1) / nb);
    const int la = std::max(0, opts.lookahead);
    T* buf = static_cast<T*>(S.buf);
    UpdateReservation reserve(p == 1 ? 32 : 0);   // the persistent panel's CUs (p = 1)
    hipStream_t ps = R.panel, us = R.update;
    const i64 kmin = std::min(m, n);
    Scratch ipiv(sizeof(i64) * std::max<i64>(kmin, 1), R.main), infos(sizeof(i64) * std::max<i64>(kt, 1), R.main);
    dzero(ipiv.p, sizeof(i64) * std::max<i64>(kmin, 1), R.main);
    dzero(infos.p, sizeof(i64) * std::max<i64>(kt, 1), R.main);
    i64* ipiv_d = ipiv.as<i64>();
    join(R.main, ps);
    join(R.main, us);
    const bool rowmajor = p == 1 && opts.lu_method != 1 && kt > 0 && env_int("SLATE_AMD_NATIVE_LU_ROWMAJOR", 1) != 0;
    if (rowmajor) {
        if (getrf_p1_rm<T>(S, la, opts.pivot_threshold, ipiv_d, infos.as<i64>(), false)) {
            dzero(ipiv.p, sizeof(i64) * std::max<i64>(kmin, 1), R.main);
            dzero(infos.p, sizeof(i64) * std::max<i64>(kt, 1), R.main);
            getrf_p1_rm<T>(S, la, opts.pivot_threshold, ipiv_d, infos.as<i64>(), true);
        }
    } else if (p == 1) {
        // ---- 1 x q: full-height panels on their owner (persistent LU
        //      panel), lookahead; models/lu.py _getrf_p1
        std::vector<std::unique_ptr<Event>> ev_tr((size_t)kt), ev_used((size_t)kt);
        // broadcast panels: a ring of NR buffers, slot k % NR rewritten at
        // step k only after the update stream finished step k - NR
        const int NR = la + 3;
        std::vector<std::unique_ptr<Scratch>> ring;
        if (q > 1)
            for (int r = 0; r < NR; ++r) ring.push_back(std::make_unique<Scratch>((size_t)m * nb * sizeof(T), ps));
        auto update_cols = [&](const T* Lp, i64 ldl, i64 r0, i64 kb, i64 c0, i64 c1, hipStream_t s) {
            if (c1 <= c0) return;
            T* cols = buf + c0 * lld;
            slate_hip::laswp_off<K<T>>(c1 - c0, kp(cols), lld, r0, r0 + kb, ipiv_d, -r0, s);
            T* Ukk = buf + r0 + c0 * lld;
            slate_hip::trsm<K<T>>('L', 'L', 'N', 'U', kb, c1 - c0, kv(T(1)), kp(Lp), ldl, kp(Ukk), lld, s);
            if (m > r0 + kb)
                gemm_k<T>('N', 'N', m - r0 - kb, c1 - c0, kb, T(-1), Lp + kb, ldl, Ukk, lld, T(1),
                          buf + r0 + kb + c0 * lld, lld, s);
        };
        for (i64 k = 0; k < kt; ++k) {
            const i64 r0 = k * nb;
            const i64 kb = std::min({nb, n - r0, m - r0});
            const i64 mk = m - r0;
            const bool own = (k % q) == pc;
            const i64 lck = tiles_before(k, q, pc) * nb;
            const i64 lc1 = std::min(tiles_before(k + 1, q, pc) * nb, nloc);
            const i64 lcla = std::min(tiles_before(k + 1 + la, q, pc) * nb, nloc);
            if (k - la - 1 >= 0) ev_tr[k - la - 1]->wait(ps);
            if (q > 1 && k >= NR) ev_used[k - NR]->wait(ps);
            T* Lb = q > 1 ? ring[k % NR]->as<T>() : nullptr;
            const T* Lp = nullptr;
            i64 ldl = mk;
            std::unique_ptr<trace_rt::Scope> sp_panel(trace_rt::g_on ? new trace_rt::Scope("getrf::panel", ps) : nullptr);
            if (own) {
                const i64 wk = std::min(nb, n - r0);
                if (opts.lu_method == 1)
                    calu_panel_1<T>(mk, wk, buf + r0 + lck * lld, lld, ipiv_d + r0, infos.as<i64>() + k,
                                    opts.pivot_threshold, opts.calu_leaf, ps);
                else
                    slate_hip::getrf_panel_ws<K<T>>(mk, wk, kp(buf + r0 + lck * lld), lld, ipiv_d + r0,
                                                    infos.as<i64>() + k, opts.pivot_threshold, false, R.lu_work, ps);
                Lp = buf + r0 + lck * lld;
                ldl = lld;
                if (q > 1) copy2d(Lb, mk, Lp, lld, mk, kb, ps);
            }
            if (q > 1) {
                gc->row->bcast(ipiv_d + r0, (size_t)kb * sizeof(i64), (int)(k % q), ps);
                gc->row->bcast(Lb, (size_t)mk * kb * sizeof(T), (int)(k % q), ps);
                Lp = Lb;
                ldl = mk;
            }
            sp_panel.reset();
            if (k >= 1 && la > 0) ev_tr[k - 1]->wait(ps);
            {
                NTRACE("getrf::lookahead", ps);
                update_cols(Lp, ldl, r0, kb, lc1, lcla, ps);
            }
            Event ev_panel;
            ev_panel.record(ps);
            ev_panel.wait(us);
            const i64 lcnx = std::max(std::min(tiles_before(k + 2 + la, q, pc) * nb, nloc), lcla);
            NTRACE("getrf::update", us);
            update_cols(Lp, ldl, r0, kb, lcla, lcnx, us);
            ev_tr[k] = std::make_unique<Event>();
            ev_tr[k]->record(us);
            update_cols(Lp, ldl, r0, kb, lcnx, nloc, us);
            if (lck > 0) slate_hip::laswp_off<K<T>>(lck, kp(buf), lld, r0, r0 + kb, ipiv_d, -r0, us);
            ev_used[k] = std::make_unique<Event>();
            ev_used[k]->record(us);
        }
        join(us, ps);
        for (auto& x : ring) x->s = ps;             // ps has joined the update stream
    } else {
        // ---- p > 1: distributed panel (rows on their owners), then per
        //      step ONE row broadcast of [my panel rows | top block |
        //      pivots] from the panel's process column, the owner-masked row
        //      exchange of every trailing column, U rows by a trsm on the top
        //      block, one GEMM (models/lu.py _getrf_general)
        Comm* colc = gc->col.get();
        Comm* rowc = gc->row.get();
        // SLATE_AMD_NATIVE_LU_XCHG=allreduce: the owner-masked all-reduce of
        // 2 kb rows x every local column per step instead of the exact moves
        static const bool p2p = [] {
            const char* e = std::getenv("SLATE_AMD_NATIVE_LU_XCHG");
            return !(e && std::strcmp(e, "allreduce") == 0);
        }();
        // panel-relative global rows of my panel rows, every step, uploaded
        // once (no host synchronisation inside the loop)
        std::vector<i64> gflat, goff((size_t)kt + 1, 0);
        for (i64 k = 0; k < kt; ++k) {
            const i64 lr_k = std::min(tiles_before(k, p, pr) * nb, mloc);
            for (i64 i = lr_k; i < mloc; ++i) gflat.push_back(l2g(i, nb, p, pr) - k * nb);
            goff[k + 1] = (i64)gflat.size();
        }
        if (gflat.empty()) gflat.push_back(0);
        Scratch gall(gflat.size() * sizeof(i64), ps);
        upload(gall.p, gflat.data(), gflat.size() * sizeof(i64), ps);
        std::vector<std::unique_ptr<Event>> ev_tr((size_t)kt);
        std::vector<std::unique_ptr<Scratch>> packs;        // step packs still read by the update stream
        if (p2p && la > 0) join(ps, us);
        for (i64 k = 0; k < kt; ++k) {
            const i64 r0 = k * nb;
            const i64 kb = std::min({nb, n - r0, m - r0});
            const int ck = (int)(k % q), rk = (int)(k % p);
            const i64 lr_k = std::min(tiles_before(k, p, pr) * nb, mloc);
            const i64 lr1 = (pr == rk) ? std::min(lr_k + kb, mloc) : lr_k;
            const i64 lck = std::min(tiles_before(k, q, pc) * nb, nloc);
            const i64 lc1 = std::min(tiles_before(k + 1, q, pc) * nb, nloc);
            const i64 nmine = mloc - lr_k;
            // pack = [L rows (nmine x kb) | T (kb x kb) | pivots (kb)]
            const size_t lbytes = (size_t)std::max<i64>(nmine, 0) * kb * sizeof(T);
            const size_t tbytes = (size_t)kb * kb * sizeof(T);
            Scratch pack(lbytes + tbytes + (size_t)kb * sizeof(i64) + 64, ps);
            T* Lp = pack.as<T>();
            T* Tt = reinterpret_cast<T*>(static_cast<char*>(pack.p) + lbytes);
            i64* pv = reinterpret_cast<i64*>(static_cast<char*>(pack.p) + lbytes + tbytes);
            std::unique_ptr<trace_rt::Scope> sp_panel(trace_rt::g_on ? new trace_rt::Scope("getrf::panel", ps) : nullptr);
            if (pc == ck) {
                if (opts.lu_method == 1)
                    calu_panel_dist<T>(S, k, kb, lck, ipiv_d, infos.as<i64>() + k, opts.pivot_threshold,
                                       opts.calu_leaf, Tt, ps);
                else
                    panel_dist<T>(S, k, kb, lck, ipiv_d, infos.as<i64>() + k, opts.pivot_threshold,
                                  opts.inner_blocking, Tt, gall.as<i64>() + goff[k], ps);
                copy2d(Lp, std::max<i64>(nmine, 1), buf + lr_k + lck * lld, lld, nmine, kb, ps);
                dcopy(pv, ipiv_d + r0, (size_t)kb * sizeof(i64), ps);
            }
            sp_panel.reset();
            NTRACE("getrf::update", ps);
            if (q > 1) rowc->bcast(pack.p, lbytes + tbytes + (size_t)kb * sizeof(i64), ck, ps);
            dcopy(ipiv_d + r0, pv, (size_t)kb * sizeof(i64), ps);
            if (p2p) {
                // exact moves: the step's pivots to the host (a wait on the
                // panel stream only: the update stream keeps running the
                // previous step's trailing GEMM meanwhile)
                std::vector<i64> hpv((size_t)kb);
                NHIP(hipMemcpyAsync(hpv.data(), pv, (size_t)kb * sizeof(i64), hipMemcpyDeviceToHost, ps));
                NHIP(hipStreamSynchronize(ps));
                const auto mv = fold_moves(hpv, r0);
                // U rows of columns [c0, c1) on the window's process row, down
                // the column over `cc`, then the GEMM -- on stream s
                auto urows = [&](i64 c0, i64 c1, Comm* cc, hipStream_t s) {
                    const i64 w = c1 - c0;
                    if (w <= 0) return;
                    Scratch Ub((size_t)kb * w * sizeof(T), s);
                    if (pr == rk) {
                        slate_hip::trsm<K<T>>('L', 'L', 'N', 'U', kb, w, kv(T(1)), kp(Tt), kb,
                                              kp(buf + lr_k + c0 * lld), lld, s);
                        copy2d(Ub.as<T>(), kb, buf + lr_k + c0 * lld, lld, kb, w, s);
                    }
                    cc->bcast(Ub.p, (size_t)kb * w * sizeof(T), rk, s);
                    if (mloc > lr1)
                        gemm_k<T>('N', 'N', mloc - lr1, w, kb, T(-1), Lp + (lr1 - lr_k), std::max<i64>(nmine, 1),
                                  Ub.as<T>(), kb, T(1), buf + lr1 + c0 * lld, lld, s);
                };
                if (la == 0) {
                    p2p_rows<T>(S, mv, {{lc1, nloc}, {0, lck}}, colc, ps);
                    urows(lc1, nloc, colc, ps);
                    continue;
                }
                // lookahead (models/lu.py _getrf_general; SLATE getrf.cc:85-235):
                // the next la tile columns on the panel stream over the column
                // communicator, the rest on the update stream over its own
                // second column communicator (two streams never share one
                // communicator); the panel of step k+1 then only waits for
                // this step's lookahead columns
                const i64 lcla = std::min(tiles_before(k + 1 + la, q, pc) * nb, nloc);
                if (k >= 1) ev_tr[k - 1]->wait(ps);        // the newest lookahead column was step k-1's trailing
                p2p_rows<T>(S, mv, {{lc1, lcla}}, colc, ps);
                urows(lc1, lcla, colc, ps);
                Event ev_la;
                ev_la.record(ps);
                ev_la.wait(us);
                packs.push_back(std::make_unique<Scratch>(0, ps));
                packs.back()->p = pack.p;                      // the pack stays alive for the update stream
                pack.p = nullptr;
                Comm* colu = gc->colu ? gc->colu.get() : colc;
                p2p_rows<T>(S, mv, {{lcla, nloc}, {0, lck}}, colu, us);
                const i64 lcnx = std::max(std::min(tiles_before(k + 2 + la, q, pc) * nb, nloc), lcla);
                urows(lcla, lcnx, colu, us);
                ev_tr[k] = std::make_unique<Event>();
                ev_tr[k]->record(us);
                urows(lcnx, nloc, colu, us);
                continue;
            }
            // every local column except the panel's own: interchanges, then
            // (trailing columns) U rows and the update
            auto trailing = [&](i64 c0, i64 c1) {
                if (c1 <= c0) return;
                Scratch plan(slate_hip::swap_plan_bytes(), ps);
                slate_hip::swap_plan(r0, r0 + kb, ipiv_d, -r0, 1, plan.p, ps);
                const i64 S2 = 2 * kb, w = c1 - c0;
                Scratch X((size_t)S2 * w * sizeof(T), ps);
                T* cols = buf + c0 * lld;
                slate_hip::xchg_gather<K<T>>(plan.p, S2, w, kp(cols), lld, kp(X.as<T>()), S2, nb, p, pr, ps);
                colc->allreduce(X.p, (size_t)S2 * w, dt_of<T>::v, 's', ps);
                slate_hip::xchg_scatter<K<T>>(plan.p, S2, w, kp(X.as<T>()), S2, kp(cols), lld, nb, p, pr, ps);
                if (c0 >= lc1) {
                    T* U = X.as<T>();
                    slate_hip::trsm<K<T>>('L', 'L', 'N', 'U', kb, w, kv(T(1)), kp(Tt), kb, kp(U), S2, ps);
                    if (pr == rk) copy2d(buf + lr_k + c0 * lld, lld, U, S2, kb, w, ps);
                    if (mloc > lr1)
                        gemm_k<T>('N', 'N', mloc - lr1, w, kb, T(-1), Lp + (lr1 - lr_k), std::max<i64>(nmine, 1), U,
                                  S2, T(1), buf + lr1 + c0 * lld, lld, ps);
                }
            };
            trailing(lc1, nloc);            // the trailing columns
            trailing(0, lck);               // the factored columns on the left
        }
        if (!packs.empty()) join(us, ps);                  // the packs are freed on ps after the update stream's last use
    }
    join(ps, R.main);
    join(us, R.main);
    std::vector<i64> h((size_t)std::max<i64>(kmin, 1));
    NHIP(hipMemcpyAsync(h.data(), ipiv_d, h.size() * sizeof(i64), hipMemcpyDeviceToHost, R.main));
    const int64_t info = read_infos(infos.as<i64>(), kt, R.main, nb);
    if (p > 1 && gc->colpeer) {
        unsigned long long e = 0;
        NHIP(hipMemcpy(&e, gc->colpeer->err, sizeof(e), hipMemcpyDeviceToHost));
        if (e) {
            gc->colpeer->dead = true;     // sticky: every later use raises instead of waiting on stale tags
            throw Error("native getrf: peer mailbox exchange timed out (a column peer never posted its record)");
        }
    }
    ipiv_out.assign((size_t)kmin, 0);
    for (i64 i = 0; i < kmin; ++i) ipiv_out[i] = h[i] + (i / nb) * nb;   // panel-relative -> global
    return reduce_info(info);
}

// op(A) = P L U: NoTrans X = U^{-1} L^{-1} P^T B; ConjTrans X = P L^{-H}
// U^{-H} B (the interchanges applied backwards at the end)
template <typename T>
int64_t getrs(Op trans, const Matrix<T>& A, const std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts) {
    Storage& SB = *B.storage();
    Runtime& R = rt();
    hipStream_t s = R.main;
    if (trans == Op::Trans && is_cplx<T>()) throw Error("native getrs: Trans of a complex matrix (use ConjTrans)");
    const i64 k = (i64)ipiv.size();
    Scratch d(sizeof(i64) * std::max<i64>(k, 1), s);
    upload(d.p, ipiv.data(), sizeof(i64) * k, s);
    Comm* colc = SB.gc->col.get();
    if (trans == Op::NoTrans) {
        permute_rows_dist<T>(SB, d.as<i64>(), 0, k, 0, SB.nloc, 1, s, colc);
        NHIP(hipStreamSynchronize(s));
        trsm<T>(Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, T(1), A, B, opts);
        trsm<T>(Side::Left, Uplo::Upper, Op::NoTrans, Diag::NonUnit, T(1), A, B, opts);
    } else {
        trsm<T>(Side::Left, Uplo::Upper, Op::ConjTrans, Diag::NonUnit, T(1), A, B, opts);
        trsm<T>(Side::Left, Uplo::Lower, Op::ConjTrans, Diag::Unit, T(1), A, B, opts);
        permute_rows_dist<T>(SB, d.as<i64>(), 0, k, 0, SB.nloc, -1, s, colc);
        NHIP(hipStreamSynchronize(s));
    }
    return 0;
}

template <typename T>
int64_t getrs(const Matrix<T>& A, const std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts) {
    return getrs<T>(Op::NoTrans, A, ipiv, B, opts);
}

template <typename T>
int64_t gesv(Matrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts) {
    const int64_t info = getrf(A, ipiv, opts);
    if (info == 0) getrs(A, ipiv, B, opts);
    return info;
}

// ------------------------------------------------------------ gemm (SUMMA)
// C = alpha A B + beta C: per k the A(:, k) block of this process row
// (row broadcast) and the B(k, :) block of this process column (column
// broadcast) -- issued on the comm stream ONE step ahead of the GEMM on the
// panel stream (double buffers, events): the broadcasts of step k+1 travel
// while GEMM k runs (SLATE gemmC's lookahead, src/gemmC.cc:104-170)
// SUMMA over the process grid: per k block, the A column block along the
// process rows and the B row block along the process columns (lookahead
// broadcasts on the comm stream), one local GEMM each.  mask: only the kept
// part of C (a stored triangle, in global coordinates) is written.
// kstruct: A's column block k / B's row block k only reach C's tiles <= k
// (1: X^H X of a lower X, X X^H of an upper X) or >= k (2: X^H X of an
// upper X): step k updates only that corner of C, so a triangular product
// costs a third of the full one (C starts at beta = 0)
template <typename T>
static void summa(T alpha, const Storage& SA, const Storage& SB, T beta, Storage& SC, const Options& opts,
                  const slate_hip::TriMask* mask, int kstruct = 0) {
    if (SA.m != SC.m || SB.n != SC.n || SA.n != SB.m) throw Error("native gemm: dimension mismatch");
    if (SA.nb != SB.nb || SA.nb != SC.nb || SA.p != SC.p || SA.q != SC.q || SB.p != SC.p || SB.q != SC.q)
        throw Error("native gemm: A, B, C must share the grid and the tile size");
    Runtime& R = rt();
    hipStream_t s = R.panel, cs = R.comm;
    join(R.main, s);
    join(R.main, cs);
    NTRACE("gemm::summa", s);
    const i64 nb = SA.nb, Kd = SA.n;
    const int p = SC.p, q = SC.q, pr = SC.pr, pc = SC.pc;
    GridComms* gc = SC.gc;
    T* Cl = static_cast<T*>(SC.buf);
    const T* Al = static_cast<const T*>(SA.buf);
    const T* Bl = static_cast<const T*>(SB.buf);
    if (kstruct) {
        if (beta != T(0)) throw Error("native summa: a triangular-structured product starts from beta = 0");
        if (SC.mloc && SC.nloc) slate_hip::geset<K<T>>('G', SC.mloc, SC.nloc, kv(T(0)), kv(T(0)), kp(Cl), SC.lld, s);
        beta = T(1);
    }
    if (p == 1 && q == 1 && !kstruct) {
        gemm_k<T>('N', 'N', SC.m, SC.n, Kd, alpha, Al, SA.lld, Bl, SB.lld, beta, Cl, SC.lld, s, mask);
    } else {
        const i64 kt = (Kd + nb - 1) / nb;
        const int la = std::max(1, opts.lookahead);
        const i64 ma = std::max<i64>(SA.mloc, 1), nbl = std::max<i64>(SB.nloc, 1);
        const int nbuf = la + 1;
        std::vector<std::unique_ptr<Scratch>> Ab, Bb;
        for (int b = 0; b < nbuf; ++b) {
            Ab.push_back(std::make_unique<Scratch>((size_t)ma * nb * sizeof(T), s));
            Bb.push_back(std::make_unique<Scratch>((size_t)nb * nbl * sizeof(T), s));
        }
        join(s, cs);                          // the buffers exist before the comm stream fills them
        std::vector<std::unique_ptr<Event>> ready((size_t)kt), used((size_t)kt);
        auto issue = [&](i64 k) {
            const int b = (int)(k % nbuf);
            const i64 kb = std::min(nb, Kd - k * nb);
            if (k >= nbuf) used[k - nbuf]->wait(cs);          // buffer b free again
            if ((int)(k % q) == pc && SA.mloc)
                copy2d(Ab[b]->as<T>(), ma, Al + tiles_before(k, q, pc) * nb * SA.lld, SA.lld, SA.mloc, kb, cs);
            if (q > 1 && SA.mloc) gc->row->bcast(Ab[b]->p, (size_t)ma * kb * sizeof(T), (int)(k % q), cs);
            if ((int)(k % p) == pr && SB.nloc)
                copy2d(Bb[b]->as<T>(), kb, Bl + tiles_before(k, p, pr) * nb, SB.lld, kb, SB.nloc, cs);
            if (p > 1 && SB.nloc) gc->col->bcast(Bb[b]->p, (size_t)kb * SB.nloc * sizeof(T), (int)(k % p), cs);
            ready[k] = std::make_unique<Event>();
            ready[k]->record(cs);
        };
        for (i64 k = 0; k < std::min<i64>(kt, la); ++k) issue(k);
        for (i64 k = 0; k < kt; ++k) {
            if (k + la < kt) issue(k + la);
            const int b = (int)(k % nbuf);
            const i64 kb = std::min(nb, Kd - k * nb);
            ready[k]->wait(s);
            i64 r0 = 0, r1 = SC.mloc, c0 = 0, c1 = SC.nloc;
            if (kstruct == 1) {
                r1 = std::min(tiles_before(k + 1, p, pr) * nb, SC.mloc);
                c1 = std::min(tiles_before(k + 1, q, pc) * nb, SC.nloc);
            } else if (kstruct == 2) {
                r0 = std::min(tiles_before(k, p, pr) * nb, SC.mloc);
                c0 = std::min(tiles_before(k, q, pc) * nb, SC.nloc);
            }
            slate_hip::TriMask mk2{};
            const slate_hip::TriMask* mp = mask;
            if (mask) {
                mk2 = *mask;
                mk2.row_off += r0;
                mk2.col_off += c0;
                mp = &mk2;
            }
            if (r1 > r0 && c1 > c0)
                gemm_k<T>('N', 'N', r1 - r0, c1 - c0, kb, alpha, Ab[b]->as<T>() + r0, ma, Bb[b]->as<T>() + c0 * kb, kb,
                          k == 0 ? beta : T(1), Cl + r0 + c0 * SC.lld, SC.lld, s, mp);
            used[k] = std::make_unique<Event>();
            used[k]->record(s);
        }
        if (kt == 0 && beta != T(1)) {
            if (mask) throw Error("native summa: k = 0 with a triangular output");
            slate_hip::gescale<K<T>>('G', SC.mloc, SC.nloc, kv(beta), kp(Cl), SC.lld, s);
        }
        for (auto& x : Ab) x->s = s;
        for (auto& x : Bb) x->s = s;
        join(cs, s);
    }
    NHIP(hipStreamSynchronize(s));
}

template <typename T>
void gemm(T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C, const Options& opts) {
    if (A.op() != Op::NoTrans || B.op() != Op::NoTrans) {
        gemm<T>(A.op(), B.op(), alpha, A.base(), B.base(), beta, C, opts);
        return;
    }
    summa<T>(alpha, *A.storage(), *B.storage(), beta, *C.storage(), opts, nullptr);
}

// op(X) as a matrix of its own (X itself for NoTrans)
template <typename T>
static Matrix<T> op_copy(Op op, const Matrix<T>& Xv) {
    // op(X) of a view X = op'(base) with op' = op composed with the view's op
    op = compose_op<T>(op, Xv.op());
    const Matrix<T> X = Xv.base();
    if (op == Op::NoTrans) return X;
    const Storage& S = *X.storage();
    Matrix<T> Y(S.n, S.m, S.nb, S.p, S.q);
    copy<T>(op, X, Y);
    return Y;
}

template <typename T>
void gemm(Op opA, Op opB, T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts) {
    const Matrix<T> Ao = op_copy<T>(opA, A);
    const Matrix<T> Bo = op_copy<T>(opB, B);
    gemm<T>(alpha, Ao, Bo, beta, C, opts);
}

// ------------------------------------------------------------ Hermitian / symmetric / triangular BLAS-3
// Reference: src/herk.cc, src/her2k.cc, src/hemm.cc (hemmA / hemmC),
// src/trmm.cc (work::trmm).  Here every one of them is the masked SUMMA
// above on operands materialised once: op(A) by the tile transpose
// exchange, a Hermitian / symmetric / triangular A expanded to a full
// matrix by two masked copies.  The output mask writes only C's stored
// triangle (herk/syrk/her2k/syr2k) and skips whole GEMM blocks above it.

// the stored triangle of C as a GEMM output mask (global coordinates)
static slate_hip::TriMask tri_mask(const Storage& S, Uplo uplo, i64 diag_off = 0) {
    slate_hip::TriMask t = lower_mask(S.nb, S.p, S.pr, S.q, S.pc, 0, 0);
    if (uplo == Uplo::Upper) t.mode = 2;
    t.diag_off = diag_off;
    return t;
}

// full matrix of a stored triangle: kind 0 = triangular (the other part
// zero; a Unit diagonal set to one), 1 = Hermitian (the other part is the
// stored one conjugate-transposed, real diagonal), 2 = symmetric
template <typename T>
Matrix<T> expand_tri(const Matrix<T>& A, Uplo uplo, int kind, Diag diag) {
    const Storage& S = *A.storage();
    if (S.m != S.n) throw Error("native: square triangular / Hermitian matrix expected");
    hipStream_t s = rt().main;
    Matrix<T> F(S.m, S.n, S.nb, S.p, S.q);
    Storage& SF = *F.storage();
    const bool unit = kind == 0 && diag == Diag::Unit;
    const slate_hip::TriMask mk = tri_mask(S, uplo, unit ? -1 : 0);
    if (S.mloc && S.nloc)
        slate_hip::gecopy_mask<K<T>>(mk, S.mloc, S.nloc, kp(static_cast<const T*>(S.buf)), S.lld,
                                     kp(static_cast<T*>(SF.buf)), SF.lld, kind == 1, s);
    if (unit) {
        const i64 nt = (S.n + S.nb - 1) / S.nb;
        for (i64 k = 0; k < nt; ++k) {
            if ((int)(k % S.p) != S.pr || (int)(k % S.q) != S.pc) continue;
            const i64 kb = std::min(S.nb, S.n - k * S.nb);
            T* d = static_cast<T*>(SF.buf) + tiles_before(k, S.p, S.pr) * S.nb +
                   tiles_before(k, S.q, S.pc) * S.nb * SF.lld;
            // diagonal tile: the part opposite the stored triangle is still
            // zero, so 'U' ('L') sets exactly the diagonal to one
            slate_hip::geset<K<T>>(uplo == Uplo::Lower ? 'U' : 'L', kb, kb, kv(T(0)), kv(T(1)), kp(d), SF.lld, s);
        }
    }
    if (kind >= 1) {
        Matrix<T> At(S.n, S.m, S.nb, S.p, S.q);
        NHIP(hipStreamSynchronize(s));
        transpose_tiles<T>(S, *At.storage(), kind == 1 ? ctrans<T>() : 'T');
        const Storage& ST = *At.storage();
        const slate_hip::TriMask mo = tri_mask(S, uplo == Uplo::Lower ? Uplo::Upper : Uplo::Lower, -1);
        // gecopy_mask zeroes what it does not keep: mask At in place, then F += At
        T* at = static_cast<T*>(ST.buf);
        if (S.mloc && S.nloc) {
            slate_hip::gecopy_mask<K<T>>(mo, S.mloc, S.nloc, kp(at), ST.lld, kp(at), ST.lld, false, s);
            slate_hip::geadd<K<T>>('G', S.mloc, S.nloc, kv(T(1)), kp(at), ST.lld, kv(T(1)),
                                   kp(static_cast<T*>(SF.buf)), SF.lld, s);
        }
    }
    NHIP(hipStreamSynchronize(s));
    return F;
}

template <typename T>
void herk(Op op, real_t<T> alpha, const Matrix<T>& A, real_t<T> beta, HermitianMatrix<T>& C, const Options& opts) {
    if (op == Op::Trans && is_cplx<T>()) throw Error("native herk: Trans of a complex matrix (use ConjTrans)");
    const Matrix<T> X = op_copy<T>(op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans, A);   // n x k
    const Matrix<T> Xh = op_copy<T>(Op::ConjTrans, X);
    const slate_hip::TriMask mk = tri_mask(*C.storage(), C.uplo());
    summa<T>(T(alpha), *X.storage(), *Xh.storage(), T(beta), *C.storage(), opts, &mk);
}

template <typename T>
void syrk(Op op, T alpha, const Matrix<T>& A, T beta, HermitianMatrix<T>& C, const Options& opts) {
    if (op == Op::ConjTrans && is_cplx<T>()) throw Error("native syrk: ConjTrans of a complex matrix (use Trans)");
    const Matrix<T> X = op_copy<T>(op == Op::NoTrans ? Op::NoTrans : Op::Trans, A);
    const Matrix<T> Xt = op_copy<T>(Op::Trans, X);
    const slate_hip::TriMask mk = tri_mask(*C.storage(), C.uplo());
    summa<T>(alpha, *X.storage(), *Xt.storage(), beta, *C.storage(), opts, &mk);
}

template <typename T>
void her2k(Op op, T alpha, const Matrix<T>& A, const Matrix<T>& B, real_t<T> beta, HermitianMatrix<T>& C,
           const Options& opts) {
    if (op == Op::Trans && is_cplx<T>()) throw Error("native her2k: Trans of a complex matrix (use ConjTrans)");
    const Op o = op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
    const Matrix<T> X = op_copy<T>(o, A), Y = op_copy<T>(o, B);
    const Matrix<T> Xh = op_copy<T>(Op::ConjTrans, X), Yh = op_copy<T>(Op::ConjTrans, Y);
    const slate_hip::TriMask mk = tri_mask(*C.storage(), C.uplo());
    summa<T>(alpha, *X.storage(), *Yh.storage(), T(beta), *C.storage(), opts, &mk);
    summa<T>(conj_of(alpha), *Y.storage(), *Xh.storage(), T(1), *C.storage(), opts, &mk);
}

template <typename T>
void syr2k(Op op, T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, HermitianMatrix<T>& C,
           const Options& opts) {
    if (op == Op::ConjTrans && is_cplx<T>()) throw Error("native syr2k: ConjTrans of a complex matrix (use Trans)");
    const Op o = op == Op::NoTrans ? Op::NoTrans : Op::Trans;
    const Matrix<T> X = op_copy<T>(o, A), Y = op_copy<T>(o, B);
    const Matrix<T> Xt = op_copy<T>(Op::Trans, X), Yt = op_copy<T>(Op::Trans, Y);
    const slate_hip::TriMask mk = tri_mask(*C.storage(), C.uplo());
    summa<T>(alpha, *X.storage(), *Yt.storage(), beta, *C.storage(), opts, &mk);
    summa<T>(alpha, *Y.storage(), *Xt.storage(), T(1), *C.storage(), opts, &mk);
}

template <typename T>
static void xmm(Side side, int kind, T alpha, const HermitianMatrix<T>& A, const Matrix<T>& B, T beta,
                Matrix<T>& C, const Options& opts) {
    const Matrix<T> Af = expand_tri<T>(A, A.uplo(), kind);
    if (side == Side::Left) summa<T>(alpha, *Af.storage(), *B.storage(), beta, *C.storage(), opts, nullptr);
    else summa<T>(alpha, *B.storage(), *Af.storage(), beta, *C.storage(), opts, nullptr);
}

template <typename T>
void hemm(Side side, T alpha, const HermitianMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts) {
    xmm<T>(side, 1, alpha, A, B, beta, C, opts);
}

template <typename T>
void symm(Side side, T alpha, const HermitianMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts) {
    xmm<T>(side, 2, alpha, A, B, beta, C, opts);
}

// B = alpha op(A) B (Left) or alpha B op(A) (Right), A triangular
template <typename T>
void trmm(Side side, Uplo uplo, Op op, Diag diag, T alpha, const Matrix<T>& Av, Matrix<T>& B, const Options& opts) {
    op = compose_op<T>(op, Av.op());
    const Matrix<T> A = Av.base();
    if (op == Op::Trans && is_cplx<T>()) throw Error("native trmm: Trans of a complex matrix (use ConjTrans)");
    const Matrix<T> Af = expand_tri<T>(A, uplo, 0, diag);
    const Matrix<T> Ao = op_copy<T>(op, Af);
    const Storage& SB = *B.storage();
    Matrix<T> W(SB.m, SB.n, SB.nb, SB.p, SB.q);
    if (side == Side::Left) summa<T>(alpha, *Ao.storage(), SB, T(0), *W.storage(), opts, nullptr);
    else summa<T>(alpha, SB, *Ao.storage(), T(0), *W.storage(), opts, nullptr);
    copy<T>(Op::NoTrans, W, B);
}

// norms of the structured matrices (src/norm.cc: henorm / synorm / trnorm):
// the stored triangle expanded to the full matrix, then the general norm
template <typename T>
double norm(Norm kind, const HermitianMatrix<T>& A) {
    return norm<T>(kind, expand_tri<T>(A, A.uplo(), 1));
}
template <typename T>
double norm_symmetric(Norm kind, const HermitianMatrix<T>& A) {
    return norm<T>(kind, expand_tri<T>(A, A.uplo(), 2));
}
template <typename T>
double norm_triangular(Norm kind, Uplo uplo, Diag diag, const Matrix<T>& A) {
    return norm<T>(kind, expand_tri<T>(A, uplo, 0, diag));
}

// ------------------------------------------------------------ aux (src/add.cc, src/set.cc)
// B = alpha A + beta B (same grid): one local kernel
template <typename T>
void add(T alpha, const Matrix<T>& Av, T beta, Matrix<T>& B) {
    const Matrix<T> A = op_copy<T>(Op::NoTrans, Av);     // a view is materialised once
    const Storage& SA = *A.storage();
    const Storage& SB = *B.storage();
    if (SA.m != SB.m || SA.n != SB.n || SA.nb != SB.nb || SA.p != SB.p || SA.q != SB.q)
        throw Error("native add: A and B must share shape, grid and nb");
    hipStream_t s = rt().main;
    if (SB.mloc && SB.nloc)
        slate_hip::geadd<K<T>>('G', SB.mloc, SB.nloc, kv(alpha), kp(static_cast<const T*>(SA.buf)), SA.lld, kv(beta),
                               kp(static_cast<T*>(SB.buf)), SB.lld, s);
    NHIP(hipStreamSynchronize(s));
}

// A = offdiag off the global diagonal, diag on it
template <typename T>
void set(T offdiag, T diag, Matrix<T>& A) {
    const Storage& S = *A.storage();
    hipStream_t s = rt().main;
    T* a = static_cast<T*>(S.buf);
    if (S.mloc && S.nloc) slate_hip::geset<K<T>>('G', S.mloc, S.nloc, kv(offdiag), kv(offdiag), kp(a), S.lld, s);
    const i64 nt = (std::min(S.m, S.n) + S.nb - 1) / S.nb;
    for (i64 k = 0; k < nt; ++k) {
        if ((int)(k % S.p) != S.pr || (int)(k % S.q) != S.pc) continue;
        const i64 mb = std::min(S.nb, S.m - k * S.nb), nbk = std::min(S.nb, S.n - k * S.nb);
        T* d = a + tiles_before(k, S.p, S.pr) * S.nb + tiles_before(k, S.q, S.pc) * S.nb * S.lld;
        slate_hip::geset<K<T>>('G', mb, nbk, kv(offdiag), kv(diag), kp(d), S.lld, s);
    }
    NHIP(hipStreamSynchronize(s));
}

// ------------------------------------------------------------ inverses
// Reference: src/potri.cc (trtri + trtrm), src/getri.cc.  Here the inverse
// is the solve against the identity with the existing factors (potrs /
// getrs: two triangular solves over n right-hand sides on the grid),
// written back over the factors.

// n x n identity on A's grid
template <typename T>
static Matrix<T> identity_like(const Storage& S) {
    Matrix<T> I(S.n, S.n, S.nb, S.p, S.q);
    Storage& SI = *I.storage();
    hipStream_t s = rt().main;
    const i64 nt = (S.n + S.nb - 1) / S.nb;
    for (i64 k = 0; k < nt; ++k) {
        if ((int)(k % S.p) != S.pr || (int)(k % S.q) != S.pc) continue;
        const i64 kb = std::min(S.nb, S.n - k * S.nb);
        T* d = static_cast<T*>(SI.buf) + tiles_before(k, S.p, S.pr) * S.nb + tiles_before(k, S.q, S.pc) * S.nb * SI.lld;
        slate_hip::geset<K<T>>('G', kb, kb, kv(T(0)), kv(T(1)), kp(d), SI.lld, s);
    }
    NHIP(hipStreamSynchronize(s));
    return I;
}

// A^-1 from the Cholesky factor in A (potrf first); the stored triangle
// of A receives the inverse.  src/potri.cc's trtri + trtrm: X = L^{-1} by
// the tile-triangular forward solve of the identity (n^3 / 3 flops), then
// A^{-1} = X^H X by the K-structured masked SUMMA (n^3 / 3) -- Upper: X =
// U^{-1}, A^{-1} = X X^H.
template <typename T>
int64_t potri(HermitianMatrix<T>& A, const Options& opts) {
    const Storage& S = *A.storage();
    const bool lower = A.uplo() == Uplo::Lower;
    Matrix<T> X = identity_like<T>(S);
    NHIP(hipStreamSynchronize(rt().main));
    trsm_left<T>(lower ? 'L' : 'U', 'N', T(1), S, *X.storage(), lower ? 1 : 2);
    const Matrix<T> Xh = op_copy<T>(Op::ConjTrans, X);
    Matrix<T> C(S.n, S.n, S.nb, S.p, S.q);
    const slate_hip::TriMask mk = tri_mask(S, A.uplo());
    if (lower) summa<T>(T(1), *Xh.storage(), *X.storage(), T(0), *C.storage(), opts, &mk, 1);
    else summa<T>(T(1), *X.storage(), *Xh.storage(), T(0), *C.storage(), opts, &mk, 1);
    hipStream_t s = rt().main;
    const Storage& SC = *C.storage();
    // stored triangle <- C (real diagonal), the other triangle of A untouched
    if (S.mloc && S.nloc)
        slate_hip::gecopy_mask_merge<K<T>>(mk, S.mloc, S.nloc, kp(static_cast<const T*>(SC.buf)), SC.lld,
                                           kp(static_cast<T*>(S.buf)), S.lld, s);
    NHIP(hipStreamSynchronize(s));
    return 0;
}

// A^-1 from the LU factors in A and ipiv (getrf first), over A: P A = L U,
// so A^-1 = U^{-1} L^{-1} P -- X = L^{-1} by the tile-triangular solve of the
// identity (n^3 / 3 flops), X = U^{-1} X (n^3), then the columns of X move
// to their permuted places inside each process row (one exchange on the row
// communicator).  Reference: src/getri.cc (trtri + trsm + column swaps).
template <typename T>
int64_t getri(Matrix<T>& A, const std::vector<int64_t>& ipiv, const Options& opts) {
    Storage& S = *A.storage();
    if (S.m != S.n) throw Error("native getri: square matrix");
    (void)opts;
    const i64 n = S.n, nb = S.nb;
    const int q = S.q, pc = S.pc;
    Matrix<T> X = identity_like<T>(S);
    Storage& SX = *X.storage();
    NHIP(hipStreamSynchronize(rt().main));
    trsm_left<T>('L', 'U', T(1), S, SX, 1);
    trsm_left<T>('U', 'N', T(1), S, SX, 0);
    // (P A)(i, :) = A(v[i], :)  =>  A^{-1}(:, v[i]) = X(:, i)
    std::vector<i64> v((size_t)n), w((size_t)n);
    for (i64 i = 0; i < n; ++i) v[i] = i;
    for (i64 i = 0; i < (i64)ipiv.size() && i < n; ++i) std::swap(v[i], v[ipiv[i]]);
    for (i64 i = 0; i < n; ++i) w[v[i]] = i;
    auto owner = [&](i64 g) { return (int)((g / nb) % q); };
    auto local = [&](i64 g) { return (g / nb / q) * nb + g % nb; };
    hipStream_t s = rt().main;
    const i64 m = S.mloc;
    const size_t es = sizeof(T);
    // destination columns of this rank grouped by the source's process column
    // (each list in increasing destination order -- the sender packs the same order)
    std::vector<std::vector<i64>> rd((size_t)q), rs((size_t)q), sd((size_t)q), ss((size_t)q);
    for (i64 lc = 0; lc < S.nloc; ++lc) {
        const i64 j = l2g(lc, nb, q, pc), i = w[j];
        rd[owner(i)].push_back(lc);
        rs[owner(i)].push_back(local(i));
    }
    for (i64 j = 0; j < n; ++j) {          // what this rank sends: sources it owns, by destination
        const i64 i = w[j];
        if (owner(i) == pc && owner(j) != pc) ss[owner(j)].push_back(local(i));
    }
    if (m > 0 && !rd[pc].empty())
        copy_cols(S.buf, S.lld, rd[pc].data(), SX.buf, SX.lld, rs[pc].data(), m, es, (i64)rd[pc].size(), s);
    if (q > 1 && m > 0) {
        std::vector<std::unique_ptr<Scratch>> bufs;
        std::vector<P2P> ops;
        std::vector<std::pair<int, Scratch*>> unpack;
        for (int d = 0; d < q; ++d) {
            if (d == pc || ss[d].empty()) continue;
            bufs.push_back(std::make_unique<Scratch>(es * m * ss[d].size(), s));
            std::vector<i64> seq(ss[d].size());
            for (size_t c = 0; c < seq.size(); ++c) seq[c] = (i64)c;
            copy_cols(bufs.back()->p, m, seq.data(), SX.buf, SX.lld, ss[d].data(), m, es, (i64)seq.size(), s);
            ops.push_back({true, d, bufs.back()->p, es * m * ss[d].size()});
        }
        for (int src = 0; src < q; ++src) {
            if (src == pc || rd[src].empty()) continue;
            bufs.push_back(std::make_unique<Scratch>(es * m * rd[src].size(), s));
            ops.push_back({false, src, bufs.back()->p, es * m * rd[src].size()});
            unpack.emplace_back(src, bufs.back().get());
        }
        if (!ops.empty()) S.gc->row->exchange(ops, s);
        for (auto& u : unpack) {
            std::vector<i64> seq(rd[u.first].size());
            for (size_t c = 0; c < seq.size(); ++c) seq[c] = (i64)c;
            copy_cols(S.buf, S.lld, rd[u.first].data(), u.second->p, m, seq.data(), m, es, (i64)seq.size(), s);
        }
    }
    NHIP(hipStreamSynchronize(s));
    return 0;
}

// ------------------------------------------------------------ trtri / trtrm (src/trtri.cc, src/trtrm.cc)
// A^{-1} of the stored triangle: the tile-triangular solve of the identity
// (n^3 / 3 flops), written back over the triangle (the other part of A and,
// for Unit, its diagonal untouched)
template <typename T>
int64_t trtri(Uplo uplo, Diag diag, Matrix<T>& A, const Options& opts) {
    (void)opts;
    Storage& S = *A.storage();
    if (S.m != S.n) throw Error("native trtri: square matrix");
    const bool lower = uplo == Uplo::Lower;
    Matrix<T> X = identity_like<T>(S);
    NHIP(hipStreamSynchronize(rt().main));
    trsm_left<T>(lower ? 'L' : 'U', diag == Diag::Unit ? 'U' : 'N', T(1), S, *X.storage(), lower ? 1 : 2);
    const slate_hip::TriMask mk = tri_mask(S, uplo, diag == Diag::Unit ? -1 : 0);
    hipStream_t s = rt().main;
    if (S.mloc && S.nloc)
        slate_hip::gecopy_mask_merge<K<T>>(mk, S.mloc, S.nloc, kp(static_cast<const T*>(X.storage()->buf)),
                                           X.storage()->lld, kp(static_cast<T*>(S.buf)), S.lld, s);
    NHIP(hipStreamSynchronize(s));
    return 0;
}

// stored triangle <- L^H L (Lower) or U U^H (Upper): the K-structured
// masked SUMMA (n^3 / 3 flops)
template <typename T>
void trtrm(Uplo uplo, Matrix<T>& A, const Options& opts) {
    Storage& S = *A.storage();
    if (S.m != S.n) throw Error("native trtrm: square matrix");
    const bool lower = uplo == Uplo::Lower;
    const Matrix<T> X = expand_tri<T>(A, uplo, 0);
    const Matrix<T> Xh = op_copy<T>(Op::ConjTrans, X);
    Matrix<T> C(S.n, S.n, S.nb, S.p, S.q);
    const slate_hip::TriMask mk = tri_mask(S, uplo);
    if (lower) summa<T>(T(1), *Xh.storage(), *X.storage(), T(0), *C.storage(), opts, &mk, 1);
    else summa<T>(T(1), *X.storage(), *Xh.storage(), T(0), *C.storage(), opts, &mk, 1);
    hipStream_t s = rt().main;
    if (S.mloc && S.nloc)
        slate_hip::gecopy_mask_merge<K<T>>(mk, S.mloc, S.nloc, kp(static_cast<const T*>(C.storage()->buf)),
                                           C.storage()->lld, kp(static_cast<T*>(S.buf)), S.lld, s);
    NHIP(hipStreamSynchronize(s));
}

// ------------------------------------------------------------ LU without pivoting (src/getrf_nopiv.cc)
// the partial-pivoting driver with a zero pivot threshold: every panel keeps
// its diagonal (no row ever moves), ipiv is the identity
template <typename T>
int64_t getrf_nopiv(Matrix<T>& A, const Options& opts) {
    Options o = opts;
    o.pivot_threshold = 0.0;
    std::vector<int64_t> ipiv;
    return getrf<T>(A, ipiv, o);
}

template <typename T>
int64_t gesv_nopiv(Matrix<T>& A, Matrix<T>& B, const Options& opts) {
    const int64_t info = getrf_nopiv<T>(A, opts);
    if (info == 0) {
        trsm<T>(Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, T(1), A, B, opts);
        trsm<T>(Side::Left, Uplo::Upper, Op::NoTrans, Diag::NonUnit, T(1), A, B, opts);
    }
    return info;
}

// ------------------------------------------------------------ Cholesky QR (src/cholqr.cc)
// G = A^H A (herk into the lower triangle), G = L L^H, Q = A L^{-H}, R = L^H
template <typename T>
int64_t cholqr(Matrix<T>& A, Matrix<T>& R, const Options& opts) {
    const Storage& SA = *A.storage();
    Storage& SR = *R.storage();
    if (SA.m < SA.n) throw Error("native cholqr: m >= n");
    if (SR.m != SA.n || SR.n != SA.n || SR.nb != SA.nb || SR.p != SA.p || SR.q != SA.q)
        throw Error("native cholqr: R must be n x n on A's grid");
    HermitianMatrix<T> G(Uplo::Lower, SA.n, SA.nb, SA.p, SA.q);
    herk<T>(Op::ConjTrans, real_t<T>(1), A, real_t<T>(0), G, opts);
    const int64_t info = potrf<T>(G, opts);
    if (info) return info;
    trsm<T>(Side::Right, Uplo::Lower, Op::ConjTrans, Diag::NonUnit, T(1), G, A, opts);
    copy<T>(Op::ConjTrans, G, R);
    const slate_hip::TriMask up = tri_mask(SR, Uplo::Upper);
    hipStream_t s = rt().main;
    if (SR.mloc && SR.nloc)
        slate_hip::gecopy_mask<K<T>>(up, SR.mloc, SR.nloc, kp(static_cast<const T*>(SR.buf)), SR.lld,
                                     kp(static_cast<T*>(SR.buf)), SR.lld, false, s);
    NHIP(hipStreamSynchronize(s));
    return 0;
}

// ------------------------------------------------------------ LQ (src/gelqf.cc, src/unmlq.cc)
// the QR of A^H: A = (Q_qr R)^H = R^H Q_qr^H, so L = R^H and Q = Q_qr^H; A
// receives (A^H factored)^H -- L in the lower trapezoid, the reflectors
// (conjugated) above it, LAPACK's LQ layout
template <typename T>
int64_t gelqf(Matrix<T>& A, LQFactors<T>& F, const Options& opts) {
    const Storage& S = *A.storage();
    F.At = std::make_shared<Matrix<T>>(S.n, S.m, S.nb, S.p, S.q);
    copy<T>(Op::ConjTrans, A, *F.At);
    geqrf<T>(*F.At, F.qr, opts);
    copy<T>(Op::ConjTrans, *F.At, A);
    return 0;
}

// C = op(Q) C, Q = Q_qr^H: Q C = Q_qr^H C, Q^H C = Q_qr C
template <typename T>
void unmlq(Op op, const Matrix<T>& A, const LQFactors<T>& F, Matrix<T>& C, const Options& opts) {
    (void)A;
    if (!F.At) throw Error("native unmlq: factor with gelqf first");
    if (op == Op::Trans && is_cplx<T>()) throw Error("native unmlq: Trans of a complex Q (use ConjTrans)");
    unmqr<T>(op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, *F.At, F.qr, C, opts);
}

// ------------------------------------------------------------ condition estimates
// ||A^-1||_1 by Higham's refinement of Hager's method (LAPACK lacn2; SLATE
// internal_norm1est.cc): fw(X) = A^-1 X, bw(X) = A^-H X on a distributed
// n x 1 matrix.  The O(n) vector steps run on a gathered copy that every
// rank holds identically (one all-gather of n scalars per solve), so every
// rank takes the same branch without extra broadcasts; the solves keep the
// O(n^2) work on the GPUs.
template <typename T, typename F, typename B>
static double norm1est(i64 n, i64 nb, int p, int q, F&& fw, B&& bw) {
    using Rl = real_t<T>;
    Matrix<T> X(n, 1, nb, p, q);
    std::vector<T> x((size_t)n), xin((size_t)n);
    auto put = [&] { X.from_host(x.data(), n); };
    auto get = [&] { X.to_host(x.data(), n); };
    auto sum_abs = [&] {
        double s = 0;
        for (auto& v : x) s += std::abs(v);
        return s;
    };
    for (auto& v : x) v = T(Rl(1) / Rl(n));
    xin = x;
    put();
    double est = 0;
    i64 jlast = -1;
    for (int it = 0; it < 5; ++it) {
        fw(X);
        get();
        const double ny = sum_abs();
        if (it > 0 && ny <= est) break;
        est = ny;
        for (auto& v : x) {
            const Rl a = std::abs(v);
            v = a > Rl(0) ? v / a : T(1);
        }
        put();
        bw(X);
        get();
        i64 j = 0;
        double zj = -1, dot = 0;
        for (i64 i = 0; i < n; ++i) {
            const double a = std::abs(x[i]);
            if (a > zj) { zj = a; j = i; }
            dot += (double)std::real(conj_of(x[i]) * xin[i]);
        }
        if (it > 0 && (j == jlast || zj <= dot)) break;
        jlast = j;
        std::fill(x.begin(), x.end(), T(0));
        x[j] = T(1);
        xin = x;
        put();
    }
    // alternating-sign test vector
    for (i64 i = 0; i < n; ++i) x[i] = T(Rl((i % 2 == 0 ? 1.0 : -1.0) * (1.0 + (double)i / (double)std::max<i64>(n - 1, 1))));
    put();
    fw(X);
    get();
    const double t = 2.0 * sum_abs() / (3.0 * (double)n);
    return std::max(est, t);
}

template <typename T>
double gecondest(Norm nrm, const Matrix<T>& LU, double Anorm, const Options& opts) {
    const Storage& S = *LU.storage();
    if (S.m != S.n) throw Error("native gecondest: square matrix");
    if (nrm != Norm::One && nrm != Norm::Inf) throw Error("native gecondest: One or Inf norm");
    if (S.n == 0) return 1.0;
    if (Anorm == 0) return 0.0;
    // A = P L U: ||A^-1|| = ||U^-1 L^-1|| (P does not change the 1- / inf-norm)
    auto fw = [&](Matrix<T>& X) {
        trsm<T>(Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, T(1), LU, X, opts);
        trsm<T>(Side::Left, Uplo::Upper, Op::NoTrans, Diag::NonUnit, T(1), LU, X, opts);
    };
    auto bw = [&](Matrix<T>& X) {
        trsm<T>(Side::Left, Uplo::Upper, Op::ConjTrans, Diag::NonUnit, T(1), LU, X, opts);
        trsm<T>(Side::Left, Uplo::Lower, Op::ConjTrans, Diag::Unit, T(1), LU, X, opts);
    };
    const double ainv = nrm == Norm::One ? norm1est<T>(S.n, S.nb, S.p, S.q, fw, bw)
                                         : norm1est<T>(S.n, S.nb, S.p, S.q, bw, fw);
    return ainv == 0 ? 0.0 : 1.0 / (ainv * Anorm);
}

template <typename T>
double pocondest(Norm nrm, const HermitianMatrix<T>& L, double Anorm, const Options& opts) {
    const Storage& S = *L.storage();
    if (nrm != Norm::One && nrm != Norm::Inf) throw Error("native pocondest: One or Inf norm");
    if (S.n == 0) return 1.0;
    if (Anorm == 0) return 0.0;
    auto f = [&](Matrix<T>& X) { potrs<T>(L, X, opts); };     // A^-1 = A^-H
    const double ainv = norm1est<T>(S.n, S.nb, S.p, S.q, f, f);
    return ainv == 0 ? 0.0 : 1.0 / (ainv * Anorm);
}

template <typename T>
double trcondest(Norm nrm, Uplo uplo, Diag diag, const Matrix<T>& A, const Options& opts) {
    const Storage& S = *A.storage();
    if (S.m != S.n) throw Error("native trcondest: square matrix");
    if (nrm != Norm::One && nrm != Norm::Inf) throw Error("native trcondest: One or Inf norm");
    if (S.n == 0) return 1.0;
    const double Anorm = norm_triangular<T>(nrm, uplo, diag, A);
    if (Anorm == 0) return 0.0;
    auto fw = [&](Matrix<T>& X) { trsm<T>(Side::Left, uplo, Op::NoTrans, diag, T(1), A, X, opts); };
    auto bw = [&](Matrix<T>& X) { trsm<T>(Side::Left, uplo, Op::ConjTrans, diag, T(1), A, X, opts); };
    const double ainv = nrm == Norm::One ? norm1est<T>(S.n, S.nb, S.p, S.q, fw, bw)
                                         : norm1est<T>(S.n, S.nb, S.p, S.q, bw, fw);
    return ainv == 0 ? 0.0 : 1.0 / (ainv * Anorm);
}

// ------------------------------------------------------------ mixed precision
// Reference: src/posv_mixed.cc, src/gesv_mixed.cc (LAPACK dsposv / dsgesv):
// factor in the lower precision (half the bytes, ~2x the MFMA rate), then
// iterative refinement in the working precision, R = B - A X with the
// full-precision A; fall back to the working-precision solve when the
// low-precision factorization fails or 30 steps do not converge
// (iter < 0 then, as in LAPACK).
template <typename T> struct lower_prec;
template <> struct lower_prec<double> { using type = float; };
template <> struct lower_prec<std::complex<double>> { using type = std::complex<float>; };

template <typename Hi, typename Lo>
static void convert(const Matrix<Hi>& A, Matrix<Lo>& B) {
    const Storage& SA = *A.storage();
    const Storage& SB = *B.storage();
    if (SA.m != SB.m || SA.n != SB.n || SA.nb != SB.nb || SA.p != SB.p || SA.q != SB.q)
        throw Error("native convert: same shape and grid");
    hipStream_t s = rt().main;
    if (SA.mloc && SA.nloc)
        slate_hip::gecopy<K<Hi>, K<Lo>>('G', 'N', SA.mloc, SA.nloc, kp(static_cast<const Hi*>(SA.buf)), SA.lld,
                                        kp(static_cast<Lo*>(SB.buf)), SB.lld, s);
    NHIP(hipStreamSynchronize(s));
}

// X += D (same grid)
template <typename T>
static void add_to(const Matrix<T>& D, Matrix<T>& X) {
    const Storage& SD = *D.storage();
    const Storage& SX = *X.storage();
    hipStream_t s = rt().main;
    if (SX.mloc && SX.nloc)
        slate_hip::geadd<K<T>>('G', SX.mloc, SX.nloc, kv(T(1)), kp(static_cast<const T*>(SD.buf)), SD.lld, kv(T(1)),
                               kp(static_cast<T*>(SX.buf)), SX.lld, s);
    NHIP(hipStreamSynchronize(s));
}

// shared refinement loop: solve_lo(R_lo) overwrites R_lo with op^-1 R_lo in
// the low precision; Af is the full working-precision matrix
template <typename T, typename Solve>
static bool refine(const Matrix<T>& Af, const Matrix<T>& B, Matrix<T>& X, int& iter, Solve&& solve_lo,
                   const Options& opts) {
    using Lo = typename lower_prec<T>::type;
    using Rl = real_t<T>;
    const Storage& SB = *B.storage();
    const i64 n = Af.storage()->n;
    const double eps = std::numeric_limits<Rl>::epsilon();
    const double cte = norm<T>(Norm::Max, Af) * eps * std::sqrt((double)n);
    Matrix<Lo> Rlo(SB.m, SB.n, SB.nb, SB.p, SB.q);
    convert<T, Lo>(B, Rlo);
    solve_lo(Rlo);
    convert<Lo, T>(Rlo, X);
    Matrix<T> R(SB.m, SB.n, SB.nb, SB.p, SB.q), D(SB.m, SB.n, SB.nb, SB.p, SB.q);
    const int itermax = 30;
    for (int it = 0; it <= itermax; ++it) {
        copy<T>(Op::NoTrans, B, R);
        gemm<T>(T(-1), Af, X, T(1), R, opts);                   // R = B - A X
        if (norm<T>(Norm::Max, R) <= norm<T>(Norm::Max, X) * cte) {
            iter = it;
            return true;
        }
        if (it == itermax) break;
        convert<T, Lo>(R, Rlo);
        solve_lo(Rlo);
        convert<Lo, T>(Rlo, D);
        add_to<T>(D, X);
    }
    return false;
}

template <typename T>
int64_t posv_mixed(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, const Options& opts) {
    using Lo = typename lower_prec<T>::type;
    const Storage& SA = *A.storage();
    HermitianMatrix<Lo> Al(A.uplo(), SA.n, SA.nb, SA.p, SA.q);
    convert<T, Lo>(A, Al);
    iter = 0;
    if (potrf<Lo>(Al, opts) == 0) {
        const Matrix<T> Af = expand_tri<T>(A, A.uplo(), 1);
        if (refine<T>(Af, B, X, iter, [&](Matrix<Lo>& R) { potrs<Lo>(Al, R, opts); }, opts)) return 0;
        iter = -31;
    } else {
        iter = -3;                                              // LAPACK: the low-precision factorization failed
    }
    copy<T>(Op::NoTrans, B, X);
    return posv<T>(A, X, opts);
}

template <typename T>
int64_t gesv_mixed(Matrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Matrix<T>& X, int& iter,
                   const Options& opts) {
    using Lo = typename lower_prec<T>::type;
    const Storage& SA = *A.storage();
    Matrix<Lo> Al(SA.m, SA.n, SA.nb, SA.p, SA.q);
    convert<T, Lo>(A, Al);
    iter = 0;
    if (getrf<Lo>(Al, ipiv, opts) == 0) {
        if (refine<T>(A, B, X, iter, [&](Matrix<Lo>& R) { getrs<Lo>(Al, ipiv, R, opts); }, opts)) return 0;
        iter = -31;
    } else {
        iter = -3;
    }
    copy<T>(Op::NoTrans, B, X);
    return gesv<T>(A, ipiv, X, opts);
}

// ------------------------------------------------------------ norm
template <typename T>
double norm(Norm kind, const Matrix<T>& Av) {
    using Rl = decltype(std::real(T()));
    if (Av.op() != Op::NoTrans && (kind == Norm::One || kind == Norm::Inf))
        kind = kind == Norm::One ? Norm::Inf : Norm::One;       // ||A^T||_1 = ||A||_inf
    const Matrix<T> A = Av.base();
    const Storage& S = *A.storage();
    Runtime& R = rt();
    hipStream_t s = R.main;
    const char k = (char)kind;
    const i64 nout = (k == 'F' ? 2 * S.nloc : S.nloc) + S.mloc;
    Scratch out(sizeof(Rl) * std::max<i64>(nout, 1), s);
    dzero(out.p, sizeof(Rl) * std::max<i64>(nout, 1), s);
    slate_hip::genorm<K<T>, Rl>(k, 'G', 'N', 0, S.mloc, S.nloc, kp(static_cast<const T*>(S.buf)), S.lld,
                                out.as<Rl>(), s);
    std::vector<Rl> hr((size_t)std::max<i64>(nout, 1));
    NHIP(hipMemcpyAsync(hr.data(), out.p, sizeof(Rl) * hr.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    std::vector<double> h(hr.begin(), hr.end());
    // global vectors for one / inf norms, scalars for max / fro
    std::vector<double> v;
    char op = 's';
    if (k == 'M') {
        double mx = 0;
        for (i64 j = 0; j < S.nloc; ++j) mx = (h[j] != h[j] || h[j] > mx) ? h[j] : mx;
        v = {mx};
        op = 'M';
    } else if (k == '1') {
        v.assign((size_t)S.n, 0.0);
        for (i64 j = 0; j < S.nloc; ++j) v[l2g(j, S.nb, S.q, S.pc)] = h[j];
    } else if (k == 'I') {
        v.assign((size_t)S.m, 0.0);
        for (i64 i = 0; i < S.mloc; ++i) v[l2g(i, S.nb, S.p, S.pr)] = h[S.nloc + i];
    } else {
        double scale = 0, sumsq = 1;
        for (i64 j = 0; j < S.nloc; ++j) {
            const double sc = h[2 * j], sq = h[2 * j + 1];
            if (sc > 0) {
                if (scale < sc) { sumsq = sq + sumsq * (scale / sc) * (scale / sc); scale = sc; }
                else sumsq += sq * (sc / scale) * (sc / scale);
            }
        }
        v = {scale * scale * sumsq};
    }
    if (R.size > 1 && !v.empty()) {
        Scratch d(sizeof(double) * v.size(), s);
        upload(d.p, v.data(), sizeof(double) * v.size(), s);
        world_comm()->allreduce(d.p, v.size(), DT::F64, op, s);
        NHIP(hipMemcpyAsync(v.data(), d.p, sizeof(double) * v.size(), hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
    }
    if (k == 'F') return std::sqrt(v[0]);
    double r = 0;
    for (double x : v) r = (x != x || x > r) ? x : r;
    return r;
}

// ------------------------------------------------------------ QR (1 x q)
// models/qr.py _geqrf_p1 in C++: panel on its owner (geqrf_panel_ws: the
// CholeskyQR2 / recursive MFMA panel), V and T along the process row, the
// block reflector applied as C -= V op(T) (V^H C) -- lookahead columns on
// the panel stream, the bulk on the update stream.  Reference:
// src/geqrf.cc:137-295 (1-D column distribution = its p = 1 case).
struct QRData {
    std::vector<i64> r0, kb;
    std::vector<std::shared_ptr<Scratch>> T;     // kb x kb upper factor per panel
    // p > 1 (TSQR): this rank's local reflector count km <= kb per panel (T is
    // km x km) and the tree over the stacked R factors, ks reflectors (0: no
    // tree) -- fac = [T km x km | tau km | Vh km x ks | Th ks x ks | tauh ks]
    std::vector<i64> km, ks;
};

template <typename T>
static void apply_panel(const T* V, i64 ldv, const T* Vh, const T* Tm, i64 kb, T* C, i64 ldc, i64 m, i64 n,
                        bool conjT, hipStream_t s) {
    if (m <= 0 || n <= 0 || kb <= 0) return;
    Scratch W((size_t)kb * n * sizeof(T), s);
    if (Vh) gemm_k<T>('N', 'N', kb, n, m, T(1), Vh, kb, C, ldc, T(0), W.as<T>(), kb, s);
    else gemm_k<T>(ctrans<T>(), 'N', kb, n, m, T(1), V, ldv, C, ldc, T(0), W.as<T>(), kb, s);
    slate_hip::trmm<K<T>>('L', 'U', conjT ? ctrans<T>() : 'N', 'N', kb, n, kv(T(1)), kp(Tm), kb, kp(W.as<T>()), kb,
                          s);
    gemm_k<T>('N', 'N', m, n, kb, T(-1), V, ldv, W.as<T>(), kb, T(1), C, ldc, s);
}

// C = Q_k^H C (conj) or Q_k C for this rank's rows >= tile k of one column
// range: Q_k = diag(Q_r) Q^ -- the local block reflector (V, Tk: km
// columns), then the tree on the top km rows (Vt km x ks, Th ks x ks) whose
// V^H C is one all-reduce over the process column `col`
template <typename T>
static void tsqr_apply(const T* V, i64 ldv, const T* Vhx, const T* Tk, i64 km, const T* Vt, const T* Th, i64 ks,
                       T* C, i64 ldc, i64 mr, i64 nc, bool conj, Comm* col, hipStream_t s) {
    if (nc <= 0) return;
    if (conj && km && mr) apply_panel<T>(V, ldv, Vhx, Tk, km, C, ldc, mr, nc, true, s);
    if (ks) {
        Scratch W((size_t)ks * nc * sizeof(T), s);
        if (km) gemm_k<T>(ctrans<T>(), 'N', ks, nc, km, T(1), Vt, km, C, ldc, T(0), W.as<T>(), ks, s);
        else slate_hip::geset<K<T>>('G', ks, nc, kv(T(0)), kv(T(0)), kp(W.as<T>()), ks, s);
        col->allreduce(W.p, (size_t)ks * nc, dt_of<T>::v, 's', s);
        slate_hip::trmm<K<T>>('L', 'U', conj ? ctrans<T>() : 'N', 'N', ks, nc, kv(T(1)), kp(Th), ks,
                              kp(W.as<T>()), ks, s);
        if (km) gemm_k<T>('N', 'N', km, nc, ks, T(-1), Vt, km, W.as<T>(), ks, T(1), C, ldc, s);
    }
    if (!conj && km && mr) apply_panel<T>(V, ldv, nullptr, Tk, km, C, ldc, mr, nc, false, s);
}

// p > 1 process rows: models/qr.py _geqrf_general in C++ -- the panel's
// process column runs a TSQR (local QR of each rank's panel rows, all-gather
// of the R factors, redundant QR of the stack; R^ lands over R of the rank
// owning tile k), the factors travel along the process row, every rank
// applies diag(Q_r) then the tree.  Reference: src/geqrf.cc:137-295 with
// internal_ttqrt.cc (its tree of triangle-triangle reductions).
template <typename T>
static int64_t geqrf_tsqr(Storage& S, QRFactors<T>& F, const Options& opts) {
    Runtime& R = rt();
    GridComms* gc = S.gc;
    const int p = S.p, q = S.q, pr = S.pr, pc = S.pc;
    const i64 nb = S.nb, m = S.m, n = S.n, lld = S.lld, mloc = S.mloc, nloc = S.nloc;
    const i64 kt = std::min((m + nb - 1) / nb, (n + nb - 1) / nb);
    const int la = std::max(0, opts.lookahead);
    const char ct = ctrans<T>();
    T* buf = static_cast<T*>(S.buf);
    hipStream_t ps = R.panel, us = R.update;
    Comm* colc = gc->col.get();
    Comm* colu = gc->colu.get();
    std::vector<i64> nloc_r(p);
    for (int r = 0; r < p; ++r) nloc_r[r] = numroc(m, nb, r, p);
    F.d = std::make_shared<QRData>();
    join(R.main, ps);
    join(R.main, us);
    const int NR = la + 3;
    std::vector<std::unique_ptr<Scratch>> ringV, ringH;
    for (int r = 0; r < NR; ++r) {
        ringV.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(mloc, 1) * nb * sizeof(T), ps));
        ringH.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(mloc, 1) * nb * sizeof(T), ps));
    }
    std::vector<std::unique_ptr<Event>> ev_tr((size_t)kt), ev_used((size_t)kt);
    for (i64 k = 0; k < kt; ++k) {
        const i64 r0 = k * nb;
        const i64 kb = std::min({nb, n - r0, m - r0});
        const int rk = (int)(k % p), ck = (int)(k % q);
        const i64 lr_k = std::min(tiles_before(k, p, pr) * nb, mloc);
        const i64 lc_k = std::min(tiles_before(k, q, pc) * nb, nloc);
        const i64 lc1 = std::min(tiles_before(k + 1, q, pc) * nb, nloc);
        const i64 lcla = std::min(tiles_before(k + 1 + la, q, pc) * nb, nloc);
        const i64 lcnx = std::max(std::min(tiles_before(k + 2 + la, q, pc) * nb, nloc), lcla);
        std::vector<i64> kr(p), soff(p);
        int holders = 0;
        for (int r = 0; r < p; ++r) {
            const i64 cnt = nloc_r[r] - std::min(tiles_before(k, p, r) * nb, nloc_r[r]);
            kr[r] = std::min(cnt, kb);
            holders += kr[r] > 0;
        }
        i64 tot = 0;
        for (int i = 0; i < p; ++i) {        // rk first: its top rows receive R^
            const int r = (rk + i) % p;
            soff[r] = tot;
            tot += kr[r];
        }
        const i64 ks = holders > 1 ? std::min(tot, kb) : 0;
        const i64 nmine = mloc - lr_k, km = kr[pr];
        if (k - la - 1 >= 0) ev_tr[k - la - 1]->wait(ps);
        if (k >= NR) ev_used[k - NR]->wait(ps);
        const size_t oT = 0, oTau = oT + km * km, oVt = oTau + km, oTh = oVt + km * ks, oTauh = oTh + ks * ks,
                     nfac = oTauh + ks;
        auto fac = std::make_shared<Scratch>(std::max<size_t>(nfac, 1) * sizeof(T), ps);
        T* f = fac->as<T>();
        T* V = ringV[k % NR]->as<T>();
        T* mine = buf + lr_k + lc_k * lld;
        if (pc == ck) {
            if (nmine)
                slate_hip::geqrf_panel_ws<K<T>>(nmine, kb, kp(mine), lld, kp(f + oTau), kp(f + oT), km, kp(V), nmine,
                                                R.qr_work, ps);
            if (ks) {
                Scratch Rb((size_t)kb * kb * sizeof(T), ps), allR((size_t)p * kb * kb * sizeof(T), ps);
                Scratch St((size_t)tot * kb * sizeof(T), ps), Vf((size_t)tot * ks * sizeof(T), ps);
                slate_hip::geset<K<T>>('G', kb, kb, kv(T(0)), kv(T(0)), kp(Rb.as<T>()), kb, ps);
                if (km) slate_hip::gecopy<K<T>, K<T>>('U', 'N', km, kb, kp(mine), lld, kp(Rb.as<T>()), kb, ps);
                colc->allgather(Rb.p, allR.p, (size_t)kb * kb * sizeof(T), ps);
                for (int r = 0; r < p; ++r)
                    if (kr[r])
                        slate_hip::gecopy<K<T>, K<T>>('G', 'N', kr[r], kb, kp(allR.as<T>() + (size_t)r * kb * kb), kb,
                                                      kp(St.as<T>() + soff[r]), tot, ps);
                slate_hip::geqrf_panel_ws<K<T>>(tot, kb, kp(St.as<T>()), tot, kp(f + oTauh), kp(f + oTh), ks,
                                                kp(Vf.as<T>()), tot, R.qr_work, ps);
                if (km)
                    slate_hip::gecopy<K<T>, K<T>>('G', 'N', km, ks, kp(Vf.as<T>() + soff[pr]), tot, kp(f + oVt), km,
                                                  ps);
                // R^ over R_rk; the local reflectors below the diagonal stay
                if (pr == rk) slate_hip::gecopy<K<T>, K<T>>('U', 'N', ks, kb, kp(St.as<T>()), tot, kp(mine), lld, ps);
            }
        }
        if (q > 1) {
            gc->row->bcast(f, nfac * sizeof(T), ck, ps);
            if (nmine && km) gc->row->bcast(V, (size_t)nmine * km * sizeof(T), ck, ps);
        }
        const T* Vhx = nullptr;
        if (nmine >= 4096 && km && nloc > lc1) {
            T* H = ringH[k % NR]->as<T>();
            slate_hip::gecopy<K<T>, K<T>>('G', ct, km, nmine, kp(V), nmine, kp(H), km, ps);
            Vhx = H;
        }
        auto upd = [&](i64 c0, i64 c1, Comm* cm, hipStream_t s) {
            tsqr_apply<T>(V, nmine, Vhx, f + oT, km, f + oVt, f + oTh, ks, buf + lr_k + c0 * lld, lld, nmine, c1 - c0,
                          true, cm, s);
        };
        if (k >= 1 && la > 0) ev_tr[k - 1]->wait(ps);
        // (wide matrix, last panel: the tile's columns beyond kb are trailing too)
        if (pc == ck && lc_k + kb < lc1) upd(lc_k + kb, lc1, colc, ps);
        upd(lc1, lcla, colc, ps);
        Event ev_panel;
        ev_panel.record(ps);
        ev_panel.wait(us);
        upd(lcla, lcnx, colu, us);
        ev_tr[k] = std::make_unique<Event>();
        ev_tr[k]->record(us);
        upd(lcnx, nloc, colu, us);
        ev_used[k] = std::make_unique<Event>();
        ev_used[k]->record(us);
        fac->s = us;
        F.d->r0.push_back(r0);
        F.d->kb.push_back(kb);
        F.d->km.push_back(km);
        F.d->ks.push_back(ks);
        F.d->T.push_back(fac);
    }
    join(ps, R.main);
    join(us, R.main);
    for (auto* v : {&ringV, &ringH})
        for (auto& x : *v) x->s = R.main;
    NHIP(hipStreamSynchronize(R.main));
    return 0;
}

template <typename T>
int64_t geqrf(Matrix<T>& A, QRFactors<T>& F, const Options& opts) {
    NTRACE("geqrf", nullptr);
    Storage& S = *A.storage();
    if (S.p != 1) return geqrf_tsqr<T>(S, F, opts);
    Runtime& R = rt();
    GridComms* gc = S.gc;
    const int q = S.q, pc = S.pc;
    const i64 nb = S.nb, m = S.m, n = S.n, lld = S.lld, nloc = S.nloc;
    const i64 kt = std::min((m + nb - 1) / nb, (n + nb - 1) / nb);
    const int la = std::max(0, opts.lookahead);
    const char ct = ctrans<T>();
    T* buf = static_cast<T*>(S.buf);
    hipStream_t ps = R.panel, us = R.update;
    F.d = std::make_shared<QRData>();
    join(R.main, ps);
    join(R.main, us);
    const int NR = la + 3;
    std::vector<std::unique_ptr<Scratch>> ringV, ringH;
    for (int r = 0; r < NR; ++r) {
        ringV.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(m, 1) * nb * sizeof(T), ps));
        ringH.push_back(std::make_unique<Scratch>((size_t)std::max<i64>(m, 1) * nb * sizeof(T), ps));
    }
    std::vector<std::unique_ptr<Event>> ev_tr((size_t)kt), ev_used((size_t)kt);
    for (i64 k = 0; k < kt; ++k) {
        const i64 r0 = k * nb;
        const i64 kb = std::min({nb, n - r0, m - r0});
        const i64 mk = m - r0;
        const bool own = (k % q) == pc;
        const i64 lck = tiles_before(k, q, pc) * nb;
        const i64 lc1 = std::min(tiles_before(k + 1, q, pc) * nb, nloc);
        const i64 lcla = std::min(tiles_before(k + 1 + la, q, pc) * nb, nloc);
        if (k - la - 1 >= 0) ev_tr[k - la - 1]->wait(ps);
        if (k >= NR) ev_used[k - NR]->wait(ps);
        auto Tk = std::make_shared<Scratch>((size_t)kb * kb * sizeof(T), ps);
        Scratch tau((size_t)kb * sizeof(T), ps);
        T* V = ringV[k % NR]->as<T>();
        if (own)
            slate_hip::geqrf_panel_ws<K<T>>(mk, kb, kp(buf + r0 + lck * lld), lld, kp(tau.as<T>()), kp(Tk->as<T>()),
                                            kb, kp(V), mk, R.qr_work, ps);
        if (q > 1) {
            gc->row->bcast(V, (size_t)mk * kb * sizeof(T), (int)(k % q), ps);
            gc->row->bcast(Tk->p, (size_t)kb * kb * sizeof(T), (int)(k % q), ps);
        }
        // explicit V^H for tall panels: the V^H C GEMMs run as NN
        const T* Vh = nullptr;
        if (mk >= 4096 && nloc > lc1) {
            T* H = ringH[k % NR]->as<T>();
            slate_hip::gecopy<K<T>, K<T>>('G', ct, kb, mk, kp(V), mk, kp(H), kb, ps);
            Vh = H;
        }
        if (k >= 1 && la > 0) ev_tr[k - 1]->wait(ps);
        if (own && lck + kb < lc1)
            apply_panel<T>(V, mk, Vh, Tk->as<T>(), kb, buf + r0 + (lck + kb) * lld, lld, mk, lc1 - lck - kb, true, ps);
        if (lcla > lc1) apply_panel<T>(V, mk, Vh, Tk->as<T>(), kb, buf + r0 + lc1 * lld, lld, mk, lcla - lc1, true, ps);
        Event ev_panel;
        ev_panel.record(ps);
        ev_panel.wait(us);
        const i64 lcnx = std::max(std::min(tiles_before(k + 2 + la, q, pc) * nb, nloc), lcla);
        apply_panel<T>(V, mk, Vh, Tk->as<T>(), kb, buf + r0 + lcla * lld, lld, mk, lcnx - lcla, true, us);
        ev_tr[k] = std::make_unique<Event>();
        ev_tr[k]->record(us);
        apply_panel<T>(V, mk, Vh, Tk->as<T>(), kb, buf + r0 + lcnx * lld, lld, mk, nloc - lcnx, true, us);
        ev_used[k] = std::make_unique<Event>();
        ev_used[k]->record(us);
        tau.s = us;
        F.d->r0.push_back(r0);
        F.d->kb.push_back(kb);
        F.d->km.push_back(kb);
        F.d->ks.push_back(0);
        F.d->T.push_back(Tk);
    }
    join(ps, R.main);
    join(us, R.main);
    for (auto* v : {&ringV, &ringH})
        for (auto& x : *v) x->s = R.main;
    NHIP(hipStreamSynchronize(R.main));
    return 0;
}

// C = op(Q) C, Q from geqrf (A's reflectors, F's T factors); the V of each
// panel is rebuilt from A on its owner and broadcast along the process row
template <typename T>
void unmqr(Op op, const Matrix<T>& A, const QRFactors<T>& F, Matrix<T>& C, const Options&) {
    const Storage& SA = *A.storage();
    Storage& SC = *C.storage();
    if (!F.d) throw Error("native unmqr: factor with geqrf first");
    if (SA.p != SC.p || SA.q != SC.q || SA.nb != SC.nb || SA.m != SC.m)
        throw Error("native unmqr: A and C on the same grid with m rows");
    if (op == Op::Trans && is_cplx<T>()) throw Error("native unmqr: Trans of a complex Q (use ConjTrans)");
    Runtime& R = rt();
    hipStream_t s = R.main;
    const int p = SA.p, q = SA.q, pr = SA.pr, pc = SA.pc;
    const i64 nb = SA.nb;
    const T* Abuf = static_cast<const T*>(SA.buf);
    T* Cbuf = static_cast<T*>(SC.buf);
    const i64 np = (i64)F.d->T.size();
    const bool conjT = op != Op::NoTrans;
    NHIP(hipStreamSynchronize(s));
    for (i64 i = 0; i < np; ++i) {
        const i64 k = conjT ? i : np - 1 - i;
        const i64 km = F.d->km[k], ks = F.d->ks[k];
        const i64 lr_k = std::min(tiles_before(k, p, pr) * nb, SA.mloc), mr = SA.mloc - lr_k;
        const i64 lck = tiles_before(k, q, pc) * nb;
        // the local reflectors (unit lower trapezoidal; on the rank owning
        // tile k R^ sits over them, which v_explicit never reads)
        Scratch V((size_t)std::max<i64>(mr * km, 1) * sizeof(T), s);
        if ((k % q) == pc && mr && km)
            slate_hip::v_explicit<K<T>>(mr, km, kp(Abuf + lr_k + lck * SA.lld), SA.lld, kp(V.as<T>()), mr, s);
        if (q > 1 && mr && km) SA.gc->row->bcast(V.p, (size_t)mr * km * sizeof(T), (int)(k % q), s);
        const T* f = static_cast<const T*>(F.d->T[k]->p);
        tsqr_apply<T>(V.as<T>(), mr, nullptr, f, km, f + km * km + km, f + km * km + km + km * ks, ks,
                      Cbuf + lr_k, SC.lld, mr, SC.nloc, conjT, SA.gc ? SA.gc->col.get() : nullptr, s);
    }
    NHIP(hipStreamSynchronize(s));
}

// min ||A X - B||, m >= n: A = Q R, Q^H B, R X = (Q^H B)(0:n) -- X in the top
// n rows of BX
template <typename T>
int64_t gels(Matrix<T>& A, Matrix<T>& BX, const Options& opts) {
    const Storage& SA = *A.storage();
    Storage& SB = *BX.storage();
    if (SA.m < SA.n) throw Error("native gels: m >= n (overdetermined / square) only");
    if (SB.m != SA.m || SB.nb != SA.nb || SB.p != SA.p || SB.q != SA.q)
        throw Error("native gels: BX must be m x nrhs on A's grid");
    QRFactors<T> F;
    geqrf<T>(A, F, opts);
    unmqr<T>(Op::ConjTrans, A, F, BX, opts);
    trsm_left<T>('U', 'N', T(1), SA, SB);
    return 0;
}

// ------------------------------------------------------------ instantiation
#define SLATE_NATIVE_INST(T)                                                                                   \
    template class Matrix<T>;                                                                                   \
    template int64_t potrf<T>(HermitianMatrix<T>&, const Options&);                                            \
    template int64_t potrs<T>(const HermitianMatrix<T>&, Matrix<T>&, const Options&);                          \
    template int64_t posv<T>(HermitianMatrix<T>&, Matrix<T>&, const Options&);                                 \
    template int64_t getrf<T>(Matrix<T>&, std::vector<int64_t>&, const Options&);                              \
    template int64_t getrs<T>(const Matrix<T>&, const std::vector<int64_t>&, Matrix<T>&, const Options&);      \
    template int64_t getrs<T>(Op, const Matrix<T>&, const std::vector<int64_t>&, Matrix<T>&, const Options&);  \
    template int64_t gesv<T>(Matrix<T>&, std::vector<int64_t>&, Matrix<T>&, const Options&);                   \
    template void gemm<T>(T, const Matrix<T>&, const Matrix<T>&, T, Matrix<T>&, const Options&);               \
    template void gemm<T>(Op, Op, T, const Matrix<T>&, const Matrix<T>&, T, Matrix<T>&, const Options&);       \
    template void copy<T>(Op, const Matrix<T>&, Matrix<T>&);                                                   \
    template void trsm<T>(Side, Uplo, Op, Diag, T, const Matrix<T>&, Matrix<T>&, const Options&);              \
    template double norm<T>(Norm, const Matrix<T>&);                                                         \
    template int64_t geqrf<T>(Matrix<T>&, QRFactors<T>&, const Options&);                                      \
    template void unmqr<T>(Op, const Matrix<T>&, const QRFactors<T>&, Matrix<T>&, const Options&);             \
    template int64_t gels<T>(Matrix<T>&, Matrix<T>&, const Options&);                                         \
    template int64_t trtri<T>(Uplo, Diag, Matrix<T>&, const Options&);                                        \
    template void trtrm<T>(Uplo, Matrix<T>&, const Options&);                                                 \
    template int64_t getrf_nopiv<T>(Matrix<T>&, const Options&);                                              \
    template int64_t getrf_tntpiv<T>(Matrix<T>&, std::vector<int64_t>&, const Options&);                      \
    template int64_t gesv_nopiv<T>(Matrix<T>&, Matrix<T>&, const Options&);                                   \
    template int64_t cholqr<T>(Matrix<T>&, Matrix<T>&, const Options&);                                       \
    template int64_t gelqf<T>(Matrix<T>&, LQFactors<T>&, const Options&);                                     \
    template void unmlq<T>(Op, const Matrix<T>&, const LQFactors<T>&, Matrix<T>&, const Options&);            \
    template void herk<T>(Op, real_t<T>, const Matrix<T>&, real_t<T>, HermitianMatrix<T>&, const Options&);    \
    template void syrk<T>(Op, T, const Matrix<T>&, T, HermitianMatrix<T>&, const Options&);                    \
    template void her2k<T>(Op, T, const Matrix<T>&, const Matrix<T>&, real_t<T>, HermitianMatrix<T>&,          \
                           const Options&);                                                                    \
    template void syr2k<T>(Op, T, const Matrix<T>&, const Matrix<T>&, T, HermitianMatrix<T>&, const Options&); \
    template void hemm<T>(Side, T, const HermitianMatrix<T>&, const Matrix<T>&, T, Matrix<T>&, const Options&);  \
    template void symm<T>(Side, T, const HermitianMatrix<T>&, const Matrix<T>&, T, Matrix<T>&, const Options&);  \
    template void trmm<T>(Side, Uplo, Op, Diag, T, const Matrix<T>&, Matrix<T>&, const Options&);             \
    template int64_t potri<T>(HermitianMatrix<T>&, const Options&);                                           \
    template int64_t getri<T>(Matrix<T>&, const std::vector<int64_t>&, const Options&);                        \
    template double norm<T>(Norm, const HermitianMatrix<T>&);                                                 \
    template double norm_symmetric<T>(Norm, const HermitianMatrix<T>&);                                       \
    template double norm_triangular<T>(Norm, Uplo, Diag, const Matrix<T>&);                                   \
    template void add<T>(T, const Matrix<T>&, T, Matrix<T>&);                                                 \
    template void set<T>(T, T, Matrix<T>&);                                                                   \
    template double gecondest<T>(Norm, const Matrix<T>&, double, const Options&);                             \
    template double pocondest<T>(Norm, const HermitianMatrix<T>&, double, const Options&);                    \
    template double trcondest<T>(Norm, Uplo, Diag, const Matrix<T>&, const Options&);                         \
    template Matrix<T> expand_tri<T>(const Matrix<T>&, Uplo, int, Diag);
SLATE_NATIVE_INST(float)
SLATE_NATIVE_INST(double)
SLATE_NATIVE_INST(std::complex<float>)
SLATE_NATIVE_INST(std::complex<double>)
#undef SLATE_NATIVE_INST
#define SLATE_NATIVE_MIXED(T)                                                                                  \
    template int64_t posv_mixed<T>(HermitianMatrix<T>&, Matrix<T>&, Matrix<T>&, int&, const Options&);        \
    template int64_t gesv_mixed<T>(Matrix<T>&, std::vector<int64_t>&, Matrix<T>&, Matrix<T>&, int&,          \
                                   const Options&);
SLATE_NATIVE_MIXED(double)
SLATE_NATIVE_MIXED(std::complex<double>)
#undef SLATE_NATIVE_MIXED

}  // namespace native
}  // namespace slate_amd
