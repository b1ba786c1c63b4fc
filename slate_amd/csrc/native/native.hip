// Native (Python-free) host runtime and drivers of slate_amd: see
// include/slate_amd/slate_native.hh.
//
// The step loops are the same MI355X designs as the Python drivers
// (slate_amd/models/chol.py, lu.py, blas3.py), written against the HIP
// runtime and RCCL directly:
//   * one process per GPU; RCCL world communicator from a TCP-bootstrapped
//     unique id; row / column communicators by ncclCommSplit (one per grid
//     dimension, every collective issued from the panel stream in one
//     program order on all ranks);
//   * a high-priority panel stream and a low-priority update stream per
//     process, dependencies as HIP events, no host synchronisation inside a
//     factorization (info values are read once at the end);
//   * every flop on the hand-written gfx950 kernels of csrc/hip (potrf_mc /
//     potrf_lds tile Cholesky, trsm_rlt, the persistent LU panel, the MFMA
//     GEMM with block-cyclic triangular masks).
// Reference call stacks: src/potrf.cc:22-210, src/getrf.cc:22-244,
// src/gemmC.cc:39-202 (SLATE's OpenMP task DAGs over MPI).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include "../hip/common.hpp"
#include "../hip/kernels.hpp"
#include "../hip/launchers.hpp"
#include "slate_amd/slate_native.hh"

namespace slate_amd {
namespace native {

using slate_hip::i64;

#define NHIP(x)                                                                                          \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) throw Error(std::string("HIP: ") + hipGetErrorString(e_) + " at " #x);     \
    } while (0)
#define NCCL(x)                                                                                          \
    do {                                                                                                 \
        ncclResult_t r_ = (x);                                                                           \
        if (r_ != ncclSuccess) throw Error(std::string("RCCL: ") + ncclGetErrorString(r_) + " at " #x);  \
    } while (0)

// ------------------------------------------------------------ runtime
struct GridComms {
    int p = 1, q = 1, pr = 0, pc = 0;
    ncclComm_t row = nullptr;   // same process row, ranked by pc
    ncclComm_t col = nullptr;   // same process column, ranked by pr
};

struct Runtime {
    bool up = false;
    int rank = 0, size = 1, local = 0;
    ncclComm_t world = nullptr;
    hipStream_t main = nullptr, panel = nullptr, update = nullptr, update_masked = nullptr;
    void* lu_work = nullptr;
    std::map<std::pair<int, int>, GridComms> grids;
    std::mutex mu;
};

static Runtime& rt() {
    static Runtime r;
    return r;
}

static int env_int(const char* k, int def) {
    const char* v = std::getenv(k);
    return v && *v ? std::atoi(v) : def;
}

// rank 0 serves the RCCL unique id on a TCP port; the others connect (with
// retries: ranks start in any order)
static void bootstrap(ncclUniqueId* id, int rank, int size) {
    const char* addr = std::getenv("MASTER_ADDR");
    if (!addr) addr = "127.0.0.1";
    const int port = env_int("SLATE_AMD_NATIVE_PORT", env_int("MASTER_PORT", 29500) + 1);
    if (rank == 0) {
        NCCL(ncclGetUniqueId(id));
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        sockaddr_in sa{};
        sa.sin_family = AF_INET;
        sa.sin_addr.s_addr = htonl(INADDR_ANY);
        sa.sin_port = htons((uint16_t)port);
        if (bind(fd, (sockaddr*)&sa, sizeof(sa)) != 0 || listen(fd, size) != 0)
            throw Error("native bootstrap: cannot listen on port " + std::to_string(port));
        for (int r = 1; r < size; ++r) {
            int c = accept(fd, nullptr, nullptr);
            if (c < 0) throw Error("native bootstrap: accept failed");
            size_t off = 0;
            while (off < sizeof(*id)) {
                ssize_t w = send(c, (const char*)id + off, sizeof(*id) - off, 0);
                if (w <= 0) throw Error("native bootstrap: send failed");
                off += (size_t)w;
            }
            close(c);
        }
        close(fd);
        return;
    }
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(addr, std::to_string(port).c_str(), &hints, &res) != 0 || !res)
        throw Error(std::string("native bootstrap: cannot resolve ") + addr);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
            size_t off = 0;
            while (off < sizeof(*id)) {
                ssize_t g = recv(fd, (char*)id + off, sizeof(*id) - off, 0);
                if (g <= 0) break;
                off += (size_t)g;
            }
            close(fd);
            if (off == sizeof(*id)) break;
        } else {
            close(fd);
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
            throw Error("native bootstrap: no connection to rank 0");
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    freeaddrinfo(res);
}

void initialize() {
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    if (R.up) return;
    R.rank = env_int("RANK", 0);
    R.size = env_int("WORLD_SIZE", 1);
    R.local = env_int("LOCAL_RANK", 0);
    NHIP(hipSetDevice(R.local));
    int lo = 0, hi = 0;
    NHIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    NHIP(hipStreamCreateWithFlags(&R.main, hipStreamNonBlocking));
    NHIP(hipStreamCreateWithPriority(&R.panel, hipStreamNonBlocking, hi));
    NHIP(hipStreamCreateWithPriority(&R.update, hipStreamNonBlocking, lo));
    // LU: the persistent panel runs <= 32 workgroups; its trailing update
    // leaves those CUs free (same CU mask as the Python driver, streams.py)
    {
        hipDeviceProp_t pr;
        NHIP(hipGetDeviceProperties(&pr, R.local));
        const int ncu = pr.multiProcessorCount, reserve = 32;
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int b = reserve; b < ncu; ++b) mask[b / 32] |= 1u << (b % 32);
        NHIP(hipExtStreamCreateWithCUMask(&R.update_masked, (uint32_t)mask.size(), mask.data()));
    }
    const size_t lw = slate_hip::getrf_work_bytes();
    NHIP(hipMalloc(&R.lu_work, lw));
    NHIP(hipMemset(R.lu_work, 0, lw));
    if (R.size > 1) {
        ncclUniqueId id;
        bootstrap(&id, R.rank, R.size);
        NCCL(ncclCommInitRank(&R.world, R.size, id, R.rank));
    }
    R.up = true;
}

void finalize() {
    Runtime& R = rt();
    std::lock_guard<std::mutex> g(R.mu);
    if (!R.up) return;
    (void)hipDeviceSynchronize();
    for (auto& kv : R.grids) {
        if (kv.second.row) ncclCommDestroy(kv.second.row);
        if (kv.second.col) ncclCommDestroy(kv.second.col);
    }
    R.grids.clear();
    if (R.world) ncclCommDestroy(R.world);
    R.world = nullptr;
    (void)hipFree(R.lu_work);
    for (hipStream_t s : {R.main, R.panel, R.update, R.update_masked}) (void)hipStreamDestroy(s);
    R.up = false;
}

int rank() { initialize(); return rt().rank; }
int size() { initialize(); return rt().size; }
const char* version() { return "slate_amd-native 2026.10.0"; }

// row / column communicators of a p x q column-major grid (collective:
// every rank creates the grids in the same order)
static GridComms* grid_comms(int p, int q) {
    Runtime& R = rt();
    if (p * q != R.size) throw Error("grid " + std::to_string(p) + "x" + std::to_string(q) +
                                     " does not match " + std::to_string(R.size) + " ranks");
    auto key = std::make_pair(p, q);
    auto it = R.grids.find(key);
    if (it != R.grids.end()) return &it->second;
    GridComms g;
    g.p = p; g.q = q;
    g.pr = R.rank % p;
    g.pc = R.rank / p;
    if (R.size > 1) {
        NCCL(ncclCommSplit(R.world, g.pr, g.pc, &g.row, nullptr));
        NCCL(ncclCommSplit(R.world, g.pc, g.pr, &g.col, nullptr));
    }
    return &(R.grids[key] = g);
}

// ------------------------------------------------------------ storage
static i64 numroc(i64 n, i64 nb, int iproc, int nprocs) {
    const i64 nblocks = n / nb;
    i64 num = (nblocks / nprocs) * nb;
    const i64 extra = nblocks % nprocs;
    if (iproc < extra) num += nb;
    else if (iproc == extra) num += n % nb;
    return num;
}
static inline i64 l2g(i64 l, i64 nb, int p, int pr) { return ((l / nb) * p + pr) * nb + l % nb; }
static inline i64 tiles_before(i64 t, int p, int pr) { return t > pr ? (t - pr + p - 1) / p : 0; }

struct Storage {
    i64 m = 0, n = 0, nb = 1;
    int p = 1, q = 1, pr = 0, pc = 0;
    i64 mloc = 0, nloc = 0, lld = 1;
    size_t esize = 8;
    void* buf = nullptr;
    GridComms* gc = nullptr;
    ~Storage() { if (buf) (void)hipFree(buf); }
};

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
    NHIP(hipMemsetAsync(s->buf, 0, bytes, rt().main));
    NHIP(hipStreamSynchronize(rt().main));
    s_ = s;
}
template <typename T> int64_t Matrix<T>::m() const { return s_->m; }
template <typename T> int64_t Matrix<T>::n() const { return s_->n; }
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
    Storage& s = *s_;
    slate_hip::matgen<T>((int)kind, seed, s.mloc, s.nloc, data(), s.lld, s.m, s.n, s.nb, s.p, s.pr, s.nb, s.q, s.pc,
                         0, 0, 1.0, rt().main);
    NHIP(hipStreamSynchronize(rt().main));
}

template <typename T>
void Matrix<T>::from_host(const T* A, int64_t lda) {
    Storage& s = *s_;
    std::vector<T> loc((size_t)s.lld * std::max<i64>(s.nloc, 1), T(0));
    for (i64 lj = 0; lj < s.nloc; ++lj) {
        const i64 gj = l2g(lj, s.nb, s.q, s.pc);
        for (i64 li = 0; li < s.mloc; ++li) loc[li + lj * s.lld] = A[l2g(li, s.nb, s.p, s.pr) + gj * lda];
    }
    NHIP(hipMemcpy(data(), loc.data(), loc.size() * sizeof(T), hipMemcpyHostToDevice));
}

template <typename T>
void Matrix<T>::to_host(T* A, int64_t lda) const {
    const Storage& s = *s_;
    Runtime& R = rt();
    std::vector<T> loc((size_t)s.lld * std::max<i64>(s.nloc, 1));
    NHIP(hipDeviceSynchronize());
    NHIP(hipMemcpy(loc.data(), data(), loc.size() * sizeof(T), hipMemcpyDeviceToHost));
    std::vector<T> g((size_t)s.m * s.n, T(0));
    for (i64 lj = 0; lj < s.nloc; ++lj) {
        const i64 gj = l2g(lj, s.nb, s.q, s.pc);
        for (i64 li = 0; li < s.mloc; ++li) g[l2g(li, s.nb, s.p, s.pr) + gj * s.m] = loc[li + lj * s.lld];
    }
    if (R.size > 1 && !g.empty()) {
        T* d = nullptr;
        NHIP(hipMalloc(&d, g.size() * sizeof(T)));
        NHIP(hipMemcpy(d, g.data(), g.size() * sizeof(T), hipMemcpyHostToDevice));
        NCCL(ncclAllReduce(d, d, g.size(), sizeof(T) == 8 ? ncclFloat64 : ncclFloat32, ncclSum, R.world, R.main));
        NHIP(hipStreamSynchronize(R.main));
        NHIP(hipMemcpy(g.data(), d, g.size() * sizeof(T), hipMemcpyDeviceToHost));
        NHIP(hipFree(d));
    }
    for (i64 j = 0; j < s.n; ++j)
        for (i64 i = 0; i < s.m; ++i) A[i + j * lda] = g[i + j * s.m];
}

template class Matrix<double>;
template class Matrix<float>;

// ------------------------------------------------------------ helpers
namespace {

struct Event {
    hipEvent_t e = nullptr;
    Event() { NHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming)); }
    ~Event() { if (e) (void)hipEventDestroy(e); }
    Event(const Event&) = delete;
    void record(hipStream_t s) { NHIP(hipEventRecord(e, s)); }
    void wait(hipStream_t s) const { NHIP(hipStreamWaitEvent(s, e, 0)); }
};

// one join point: stream b waits for everything issued so far on stream a
static void join(hipStream_t a, hipStream_t b) {
    Event ev;
    ev.record(a);
    ev.wait(b);
}

// device scratch freed after the owning stream reaches it (stream-ordered)
struct Scratch {
    void* p = nullptr;
    hipStream_t s = nullptr;
    Scratch(size_t bytes, hipStream_t st) : s(st) { if (bytes) NHIP(hipMallocAsync(&p, bytes, st)); }
    ~Scratch() { if (p) (void)hipFreeAsync(p, s); }
    template <typename T> T* as() { return static_cast<T*>(p); }
};

static void gemm_d(char ta, char tb, i64 m, i64 n, i64 k, double alpha, const double* A, i64 lda, const double* B,
                   i64 ldb, double beta, double* C, i64 ldc, hipStream_t s, const slate_hip::TriMask* mask = nullptr) {
    if (m <= 0 || n <= 0) return;
    slate_hip::GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = alpha; c.beta_re = beta;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    if (mask) c.mask = *mask;
    slate_hip::gemm_real<double>(c, s);
}

// lower-triangle mask of a local block whose (0, 0) is local (r0, c0) of a
// block-cyclic matrix (the Python drivers' (1, nb, p, pr, q, pc, r0, c0, 0))
static slate_hip::TriMask lower_mask(i64 nb, int p, int pr, int q, int pc, i64 r0, i64 c0) {
    slate_hip::TriMask t;
    t.mode = 1; t.nb = nb; t.p = p; t.pr = pr; t.q = q; t.pc = pc; t.row_off = r0; t.col_off = c0; t.diag_off = 0;
    return t;
}

static int64_t read_infos(const i64* d, i64 nt, hipStream_t s, i64 nb) {
    std::vector<i64> h((size_t)std::max<i64>(nt, 1));
    NHIP(hipMemcpyAsync(h.data(), d, h.size() * sizeof(i64), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    for (i64 t = 0; t < nt; ++t)
        if (h[t] > 0) return t * nb + h[t];
    return 0;
}

static int64_t reduce_info(int64_t info) {
    Runtime& R = rt();
    if (R.size == 1) return info;
    const i64 big = (i64)1 << 62;
    i64* d = nullptr;
    NHIP(hipMallocAsync(&d, sizeof(i64), R.main));
    i64 v = info > 0 ? info : big;
    NHIP(hipMemcpyAsync(d, &v, sizeof(i64), hipMemcpyHostToDevice, R.main));
    NCCL(ncclAllReduce(d, d, 1, ncclInt64, ncclMin, R.world, R.main));
    NHIP(hipMemcpyAsync(&v, d, sizeof(i64), hipMemcpyDeviceToHost, R.main));
    NHIP(hipFreeAsync(d, R.main));
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

static ColPlan rows_plan(std::vector<i64>& flat, i64 m, i64 nb, int p, int q, int pc, i64 tfirst, i64 tend,
                         i64 cols_from) {
    auto mb = [&](i64 j) { return std::min(nb, m - j * nb); };
    std::vector<i64> need;
    for (i64 j = cols_from; j < tend; ++j)
        if (j % q == pc) need.push_back(j);
    ColPlan P;
    P.off.assign(p, 0); P.cnt.assign(p, 0);
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
// of the plan's tile range, from Prow (this process row's panel rows)
static void assemble_cols(const ColPlan& P, const i64* idx, const double* Prow, i64 ldp, i64 kb, GridComms* gc,
                          double* Lcol, hipStream_t s) {
    if (P.tot == 0) return;
    Scratch R((size_t)P.tot * kb * 8, s);
    i64 pos = 0;
    for (int r = 0; r < gc->p; ++r) {
        const i64 cnt = P.cnt[r];
        if (cnt) {
            Scratch tmp((size_t)cnt * kb * 8, s);
            if (gc->pr == r) slate_hip::permute_rows_gather<double>(cnt, kb, Prow, ldp, tmp.as<double>(), cnt, idx + P.off[r], s);
            if (gc->p > 1) NCCL(ncclBroadcast(tmp.p, tmp.p, (size_t)cnt * kb, ncclFloat64, r, gc->col, s));
            NHIP(hipMemcpy2DAsync(R.as<double>() + pos, P.tot * 8, tmp.p, cnt * 8, cnt * 8, kb,
                                  hipMemcpyDeviceToDevice, s));
        }
        pos += cnt;
    }
    slate_hip::permute_rows_gather<double>(P.order_cnt, kb, R.as<double>(), P.tot, Lcol, P.order_cnt,
                                           idx + P.order_off, s);
}

}  // namespace

// ------------------------------------------------------------ potrf
// One rank owning the whole matrix: trailing update per GROUP of 2 tiles
// (K = 2 nb on the MFMA GEMM), lookahead in groups (chol.py
// _potrf_1x1_grouped).
static void potrf_1x1(double* A, i64 lda, i64 n, i64 nb, int la, i64* infos) {
    Runtime& R = rt();
    hipStream_t ps = R.panel, us = R.update;
    const i64 nt = (n + nb - 1) / nb;
    const i64 G = 2;
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
        for (i64 u = tfirst; u < tlast; ++u) {
            const i64 cu = off(u), cu1 = off(u + 1);
            if (cu > c0) {
                // the group's earlier panels -> column u (rows >= cu)
                slate_hip::TriMask mk = lower_mask(nb, 1, 0, 1, 0, cu, cu);
                gemm_d('N', 'T', n - cu, cu1 - cu, cu - c0, -1.0, A + cu + c0 * lda, lda, A + cu + c0 * lda, lda, 1.0,
                       A + cu + cu * lda, lda, ps, &mk);
            }
            slate_hip::potrf_fast((int)(cu1 - cu), A + cu + cu * lda, lda, infos + u, 0, ps);
            if (n > cu1)
                slate_hip::trsm_rlt_fast(n - cu1, cu1 - cu, 1.0, A + cu + cu * lda, lda, A + cu1 + cu * lda, lda, false,
                                         ps);
        }
        // P = A[c0:n, c0:c2]; update columns [lo, hi) (rows >= lo) on stream s
        auto update = [&](i64 lo, i64 hi, hipStream_t s) {
            if (hi <= lo) return;
            slate_hip::TriMask mk = lower_mask(nb, 1, 0, 1, 0, lo, lo);
            gemm_d('N', 'T', n - lo, hi - lo, c2 - c0, -1.0, A + lo + c0 * lda, lda, A + lo + c0 * lda, lda, 1.0,
                   A + lo + lo * lda, lda, s, &mk);
        };
        const i64 la_end = gstart(gi + 1 + la);
        if (gi >= 1 && la > 0) ev_tr[gi - 1]->wait(ps);
        update(c2, la_end, ps);
        Event ev_panel;
        ev_panel.record(ps);
        ev_panel.wait(us);
        const i64 nx_end = std::max(gstart(gi + 2 + la), la_end);
        update(la_end, nx_end, us);
        ev_tr[gi] = std::make_unique<Event>();
        ev_tr[gi]->record(us);
        update(nx_end, n, us);
    }
    join(ps, R.main);
    join(us, R.main);
}

// p x q grid (chol.py _potrf_lower without the diag-first stream): panel
// stream = tile potrf, column bcast of the diagonal tile, trsm, row bcast of
// the panel, column gathers of the transposed operand, lookahead GEMM; update
// stream = the trailing GEMMs.  Every collective on the panel stream.
static void potrf_grid(Storage& S, int la, i64* infos) {
    Runtime& R = rt();
    GridComms* gc = S.gc;
    const int p = S.p, q = S.q, pr = S.pr, pc = S.pc;
    const i64 nb = S.nb, n = S.n, lld = S.lld;
    double* buf = static_cast<double*>(S.buf);
    const i64 nt = (n + nb - 1) / nb;
    const i64 lr_end = S.mloc, lc_end = S.nloc;
    hipStream_t ps = R.panel, us = R.update;
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
    NHIP(hipMemcpyAsync(idx.p, flat.data(), flat.size() * sizeof(i64), hipMemcpyHostToDevice, ps));
    join(R.main, ps);
    join(R.main, us);
    std::vector<std::unique_ptr<Event>> ev_tr((size_t)nt);
    // buffers that the update stream reads are freed on it
    for (i64 t = 0; t < nt; ++t) {
        const i64 g = t;
        const i64 kb = std::min(nb, n - g * nb);
        const i64 lrg = tiles_before(g, p, pr) * nb, lcg = tiles_before(g, q, pc) * nb;
        const i64 lr1 = std::min(tiles_before(g + 1, p, pr) * nb, lr_end);
        const i64 lc1 = std::min(tiles_before(g + 1, q, pc) * nb, lc_end);
        const bool own_col = (g % q) == pc, own_diag = own_col && (g % p) == pr;
        if (t - la - 1 >= 0) ev_tr[t - la - 1]->wait(ps);
        if (own_diag) slate_hip::potrf_fast((int)kb, buf + lrg + lcg * lld, lld, infos + t, 0, ps);
        const i64 nrow = lr_end - lr1;
        if (own_col) {
            const double* D = buf + lrg + lcg * lld;
            i64 ldd = lld;
            Scratch Dt(p > 1 ? (size_t)kb * kb * 8 : 0, ps);
            if (p > 1) {
                if (own_diag)
                    NHIP(hipMemcpy2DAsync(Dt.p, kb * 8, buf + lrg + lcg * lld, lld * 8, kb * 8, kb,
                                          hipMemcpyDeviceToDevice, ps));
                NCCL(ncclBroadcast(Dt.p, Dt.p, (size_t)kb * kb, ncclFloat64, (int)(g % p), gc->col, ps));
                D = Dt.as<double>();
                ldd = kb;
            }
            if (nrow) slate_hip::trsm_rlt_fast(nrow, kb, 1.0, D, ldd, buf + lr1 + lcg * lld, lld, false, ps);
        }
        // panel -> row (Prow: nrow x kb, contiguous)
        auto Prow = std::make_shared<Scratch>((size_t)std::max<i64>(nrow, 1) * kb * 8, ps);
        const double* P = buf + lr1 + lcg * lld;
        i64 ldp = lld;
        if (q > 1) {
            if (own_col && nrow)
                NHIP(hipMemcpy2DAsync(Prow->p, nrow * 8, buf + lr1 + lcg * lld, lld * 8, nrow * 8, kb,
                                      hipMemcpyDeviceToDevice, ps));
            if (nrow) NCCL(ncclBroadcast(Prow->p, Prow->p, (size_t)nrow * kb, ncclFloat64, (int)(g % q), gc->row, ps));
            P = Prow->as<double>();
            ldp = nrow;
        }
        // transposed operands: lookahead tiles, then the rest
        const ColPlan& A1 = plans[t].first;
        const ColPlan& A2 = plans[t].second;
        auto Lla = std::make_shared<Scratch>((size_t)std::max<i64>(A1.order_cnt, 1) * kb * 8, ps);
        auto Lcol = std::make_shared<Scratch>((size_t)std::max<i64>(A2.order_cnt, 1) * kb * 8, ps);
        const i64* d_idx = idx.as<i64>();
        const double* La;
        i64 lda_la;
        if (p > 1 || q > 1) {
            assemble_cols(A1, d_idx, P, ldp, kb, gc, Lla->as<double>(), ps);
            La = Lla->as<double>();
            lda_la = std::max<i64>(A1.order_cnt, 1);
        } else {
            La = P;
            lda_la = ldp;
        }
        const i64 lc_la = std::min(tiles_before(g + 1 + la, q, pc) * nb, lc_end);
        if (t >= 1 && la > 0) ev_tr[t - 1]->wait(ps);
        if (lc_la > lc1 && nrow) {
            slate_hip::TriMask mk = lower_mask(nb, p, pr, q, pc, lr1, lc1);
            gemm_d('N', 'T', nrow, lc_la - lc1, kb, -1.0, P, ldp, La, lda_la, 1.0, buf + lr1 + lc1 * lld, lld, ps, &mk);
        }
        const double* Lc;
        i64 ldlc, loff;
        if (p > 1 || q > 1) {
            assemble_cols(A2, d_idx, P, ldp, kb, gc, Lcol->as<double>(), ps);
            Lc = Lcol->as<double>();
            ldlc = std::max<i64>(A2.order_cnt, 1);
            loff = lc_la;
        } else {
            Lc = P;
            ldlc = ldp;
            loff = lc1;
        }
        Event ev_panel;
        ev_panel.record(ps);
        ev_panel.wait(us);
        const i64 lc_nx = std::max(std::min(tiles_before(g + 2 + la, q, pc) * nb, lc_end), lc_la);
        for (int part = 0; part < 2; ++part) {
            const i64 c0 = part == 0 ? lc_la : lc_nx, c1 = part == 0 ? lc_nx : lc_end;
            if (c1 > c0 && nrow) {
                slate_hip::TriMask mk = lower_mask(nb, p, pr, q, pc, lr1, c0);
                gemm_d('N', 'T', nrow, c1 - c0, kb, -1.0, P, ldp, Lc + (c0 - loff), ldlc, 1.0, buf + lr1 + c0 * lld,
                       lld, us, &mk);
            }
            if (part == 0) {
                ev_tr[t] = std::make_unique<Event>();
                ev_tr[t]->record(us);
            }
        }
        // the step's operand buffers are released once the update stream is
        // past them: move their frees to the update stream
        Prow->s = us; Lla->s = us; Lcol->s = us;
        join(ps, us);      // frees on us are ordered after the panel's writes
    }
    join(ps, R.main);
    join(us, R.main);
}

int64_t potrf(HermitianMatrix<double>& A, const Options& opts) {
    if (A.uplo() != Uplo::Lower) throw Error("native potrf: Lower storage only (use the conjugate transpose)");
    Storage& S = *A.storage();
    Runtime& R = rt();
    const i64 nt = (S.n + S.nb - 1) / S.nb;
    const int la = std::max(0, opts.lookahead);
    i64* infos = nullptr;
    NHIP(hipMallocAsync(&infos, sizeof(i64) * std::max<i64>(nt, 1), R.main));
    NHIP(hipMemsetAsync(infos, 0, sizeof(i64) * std::max<i64>(nt, 1), R.main));
    if (S.p == 1 && S.q == 1 && nt > 2)
        potrf_1x1(static_cast<double*>(S.buf), S.lld, S.n, S.nb, la, infos);
    else
        potrf_grid(S, la, infos);
    const int64_t info = read_infos(infos, nt, R.main, S.nb);
    NHIP(hipFreeAsync(infos, R.main));
    return reduce_info(info);
}

// ------------------------------------------------------------ solves (one rank)
static void require_1x1(const Storage& S, const char* what) {
    if (S.p != 1 || S.q != 1)
        throw Error(std::string("native ") + what + ": 1 x 1 grids only (the Python package covers p x q)");
}

int64_t potrs(const HermitianMatrix<double>& A, Matrix<double>& B, const Options&) {
    const Storage& S = *A.storage();
    Storage& T = *B.storage();
    require_1x1(S, "potrs");
    require_1x1(T, "potrs");
    hipStream_t s = rt().main;
    const double* L = static_cast<const double*>(S.buf);
    double* X = static_cast<double*>(T.buf);
    slate_hip::trsm<double>('L', 'L', 'N', 'N', S.n, T.n, 1.0, L, S.lld, X, T.lld, s);
    slate_hip::trsm<double>('L', 'L', 'T', 'N', S.n, T.n, 1.0, L, S.lld, X, T.lld, s);
    NHIP(hipStreamSynchronize(s));
    return 0;
}

int64_t posv(HermitianMatrix<double>& A, Matrix<double>& B, const Options& opts) {
    const int64_t info = potrf(A, opts);
    if (info == 0) potrs(A, B, opts);
    return info;
}

// ------------------------------------------------------------ getrf (1 x q)
int64_t getrf(Matrix<double>& A, std::vector<int64_t>& ipiv_out, const Options& opts) {
    Storage& S = *A.storage();
    Runtime& R = rt();
    if (S.p != 1) throw Error("native getrf: 1 x q grids (the Python package covers p x q)");
    GridComms* gc = S.gc;
    const int q = S.q, pc = S.pc;
    const i64 nb = S.nb, m = S.m, n = S.n, lld = S.lld, nloc = S.nloc;
    const i64 kt = std::min((m + nb - 1) / nb, (n + nb - 1) / nb);
    const int la = std::max(0, opts.lookahead);
    double* buf = static_cast<double*>(S.buf);
    hipStream_t ps = R.panel, us = R.update_masked;
    const i64 kmin = std::min(m, n);
    i64 *ipiv = nullptr, *infos = nullptr;
    NHIP(hipMallocAsync(&ipiv, sizeof(i64) * std::max<i64>(kmin, 1), R.main));
    NHIP(hipMallocAsync(&infos, sizeof(i64) * std::max<i64>(kt, 1), R.main));
    NHIP(hipMemsetAsync(ipiv, 0, sizeof(i64) * std::max<i64>(kmin, 1), R.main));
    NHIP(hipMemsetAsync(infos, 0, sizeof(i64) * std::max<i64>(kt, 1), R.main));
    join(R.main, ps);
    join(R.main, us);
    std::vector<std::unique_ptr<Event>> ev_tr((size_t)kt);
    // apply step k (pivots, U-row trsm, GEMM) to local columns [c0, c1)
    auto update_cols = [&](const double* Lp, i64 ldl, i64 r0, i64 kb, i64 c0, i64 c1, hipStream_t s) {
        if (c1 <= c0) return;
        double* cols = buf + c0 * lld;
        slate_hip::laswp_off<double>(c1 - c0, cols, lld, r0, r0 + kb, ipiv, -r0, s);
        double* Ukk = buf + r0 + c0 * lld;
        slate_hip::trsm<double>('L', 'L', 'N', 'U', kb, c1 - c0, 1.0, Lp, ldl, Ukk, lld, s);
        if (m > r0 + kb) gemm_d('N', 'N', m - r0 - kb, c1 - c0, kb, -1.0, Lp + kb, ldl, Ukk, lld, 1.0,
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
        auto Lbuf = std::make_shared<Scratch>(own && q == 1 ? 0 : (size_t)mk * kb * 8, ps);
        const double* Lp;
        i64 ldl;
        if (own) {
            const i64 wk = std::min(nb, n - r0);
            slate_hip::getrf_panel_ws<double>(mk, wk, buf + r0 + lck * lld, lld, ipiv + r0, infos + k,
                                              opts.pivot_threshold, false, R.lu_work, ps);
            Lp = buf + r0 + lck * lld;
            ldl = lld;
            if (q > 1)
                NHIP(hipMemcpy2DAsync(Lbuf->p, mk * 8, Lp, lld * 8, mk * 8, kb, hipMemcpyDeviceToDevice, ps));
        }
        if (q > 1) {
            NCCL(ncclBroadcast(ipiv + r0, ipiv + r0, (size_t)kb, ncclInt64, (int)(k % q), gc->row, ps));
            NCCL(ncclBroadcast(Lbuf->p, Lbuf->p, (size_t)mk * kb, ncclFloat64, (int)(k % q), gc->row, ps));
            Lp = Lbuf->as<double>();
            ldl = mk;
        }
        if (k >= 1 && la > 0) ev_tr[k - 1]->wait(ps);
        update_cols(Lp, ldl, r0, kb, lc1, lcla, ps);
        Event ev_panel;
        ev_panel.record(ps);
        ev_panel.wait(us);
        const i64 lcnx = std::max(std::min(tiles_before(k + 2 + la, q, pc) * nb, nloc), lcla);
        update_cols(Lp, ldl, r0, kb, lcla, lcnx, us);
        ev_tr[k] = std::make_unique<Event>();
        ev_tr[k]->record(us);
        update_cols(Lp, ldl, r0, kb, lcnx, nloc, us);
        if (lck > 0) slate_hip::laswp_off<double>(lck, buf, lld, r0, r0 + kb, ipiv, -r0, us);
        Lbuf->s = us;
        join(ps, us);
    }
    join(ps, R.main);
    join(us, R.main);
    std::vector<i64> h((size_t)std::max<i64>(kmin, 1));
    NHIP(hipMemcpyAsync(h.data(), ipiv, h.size() * sizeof(i64), hipMemcpyDeviceToHost, R.main));
    const int64_t info = read_infos(infos, kt, R.main, nb);
    NHIP(hipFreeAsync(ipiv, R.main));
    NHIP(hipFreeAsync(infos, R.main));
    NHIP(hipStreamSynchronize(R.main));
    ipiv_out.assign((size_t)kmin, 0);
    for (i64 i = 0; i < kmin; ++i) ipiv_out[i] = h[i] + (i / nb) * nb;   // panel-relative -> global
    return reduce_info(info);
}

int64_t getrs(const Matrix<double>& A, const std::vector<int64_t>& ipiv, Matrix<double>& B, const Options&) {
    const Storage& S = *A.storage();
    Storage& T = *B.storage();
    require_1x1(S, "getrs");
    require_1x1(T, "getrs");
    hipStream_t s = rt().main;
    const i64 k = (i64)ipiv.size();
    i64* d = nullptr;
    NHIP(hipMallocAsync(&d, sizeof(i64) * std::max<i64>(k, 1), s));
    NHIP(hipMemcpyAsync(d, ipiv.data(), sizeof(i64) * k, hipMemcpyHostToDevice, s));
    double* X = static_cast<double*>(T.buf);
    slate_hip::laswp_off<double>(T.n, X, T.lld, 0, k, d, 0, s);
    const double* F = static_cast<const double*>(S.buf);
    slate_hip::trsm<double>('L', 'L', 'N', 'U', S.n, T.n, 1.0, F, S.lld, X, T.lld, s);
    slate_hip::trsm<double>('L', 'U', 'N', 'N', S.n, T.n, 1.0, F, S.lld, X, T.lld, s);
    NHIP(hipFreeAsync(d, s));
    NHIP(hipStreamSynchronize(s));
    return 0;
}

int64_t gesv(Matrix<double>& A, std::vector<int64_t>& ipiv, Matrix<double>& B, const Options& opts) {
    const int64_t info = getrf(A, ipiv, opts);
    if (info == 0) getrs(A, ipiv, B, opts);
    return info;
}

// ------------------------------------------------------------ gemm (SUMMA)
void gemm(double alpha, const Matrix<double>& A, const Matrix<double>& B, double beta, Matrix<double>& C,
          const Options&) {
    const Storage& SA = *A.storage();
    const Storage& SB = *B.storage();
    Storage& SC = *C.storage();
    if (SA.m != SC.m || SB.n != SC.n || SA.n != SB.m) throw Error("native gemm: dimension mismatch");
    if (SA.nb != SB.nb || SA.nb != SC.nb || SA.p != SC.p || SA.q != SC.q || SB.p != SC.p || SB.q != SC.q)
        throw Error("native gemm: A, B, C must share the grid and the tile size");
    Runtime& R = rt();
    hipStream_t s = R.panel;
    join(R.main, s);
    const i64 nb = SA.nb, K = SA.n;
    const int p = SC.p, q = SC.q, pr = SC.pr, pc = SC.pc;
    GridComms* gc = SC.gc;
    double* Cl = static_cast<double*>(SC.buf);
    const double* Al = static_cast<const double*>(SA.buf);
    const double* Bl = static_cast<const double*>(SB.buf);
    if (p == 1 && q == 1) {
        gemm_d('N', 'N', SC.m, SC.n, K, alpha, Al, SA.lld, Bl, SB.lld, beta, Cl, SC.lld, s);
    } else {
        const i64 kt = (K + nb - 1) / nb;
        for (i64 k = 0; k < kt; ++k) {
            const i64 kb = std::min(nb, K - k * nb);
            // A(:, k): this process row's rows, from process column k % q
            Scratch Ak((size_t)std::max<i64>(SA.mloc, 1) * kb * 8, s);
            if ((int)(k % q) == pc && SA.mloc)
                NHIP(hipMemcpy2DAsync(Ak.p, SA.mloc * 8, Al + tiles_before(k, q, pc) * nb * SA.lld, SA.lld * 8,
                                      SA.mloc * 8, kb, hipMemcpyDeviceToDevice, s));
            if (q > 1 && SA.mloc)
                NCCL(ncclBroadcast(Ak.p, Ak.p, (size_t)SA.mloc * kb, ncclFloat64, (int)(k % q), gc->row, s));
            // B(k, :): this process column's columns, from process row k % p
            Scratch Bk((size_t)kb * std::max<i64>(SB.nloc, 1) * 8, s);
            if ((int)(k % p) == pr && SB.nloc)
                NHIP(hipMemcpy2DAsync(Bk.p, kb * 8, Bl + tiles_before(k, p, pr) * nb, SB.lld * 8, kb * 8, SB.nloc,
                                      hipMemcpyDeviceToDevice, s));
            if (p > 1 && SB.nloc)
                NCCL(ncclBroadcast(Bk.p, Bk.p, (size_t)kb * SB.nloc, ncclFloat64, (int)(k % p), gc->col, s));
            gemm_d('N', 'N', SC.mloc, SC.nloc, kb, alpha, Ak.as<double>(), std::max<i64>(SA.mloc, 1),
                   Bk.as<double>(), kb, k == 0 ? beta : 1.0, Cl, SC.lld, s);
        }
        if (kt == 0 && beta != 1.0)
            slate_hip::gescale<double>('G', SC.mloc, SC.nloc, beta, Cl, SC.lld, s);
    }
    NHIP(hipStreamSynchronize(s));
}

// ------------------------------------------------------------ norm
double norm(Norm kind, const Matrix<double>& A) {
    const Storage& S = *A.storage();
    Runtime& R = rt();
    hipStream_t s = R.main;
    const char k = (char)kind;
    const i64 nout = (k == 'F' ? 2 * S.nloc : S.nloc) + S.mloc;
    double* out = nullptr;
    NHIP(hipMallocAsync(&out, sizeof(double) * std::max<i64>(nout, 1), s));
    NHIP(hipMemsetAsync(out, 0, sizeof(double) * std::max<i64>(nout, 1), s));
    slate_hip::genorm<double, double>(k, 'G', 'N', 0, S.mloc, S.nloc, static_cast<const double*>(S.buf), S.lld, out,
                                      s);
    std::vector<double> h((size_t)std::max<i64>(nout, 1));
    NHIP(hipMemcpyAsync(h.data(), out, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipFreeAsync(out, s));
    NHIP(hipStreamSynchronize(s));
    // global vectors for one / inf norms, scalars for max / fro
    std::vector<double> v;
    ncclRedOp_t op = ncclSum;
    if (k == 'M') {
        double mx = 0;
        for (i64 j = 0; j < S.nloc; ++j) mx = (h[j] != h[j] || h[j] > mx) ? h[j] : mx;
        v = {mx};
        op = ncclMax;
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
        double* d = nullptr;
        NHIP(hipMallocAsync(&d, sizeof(double) * v.size(), s));
        NHIP(hipMemcpyAsync(d, v.data(), sizeof(double) * v.size(), hipMemcpyHostToDevice, s));
        NCCL(ncclAllReduce(d, d, v.size(), ncclFloat64, op, R.world, s));
        NHIP(hipMemcpyAsync(v.data(), d, sizeof(double) * v.size(), hipMemcpyDeviceToHost, s));
        NHIP(hipFreeAsync(d, s));
        NHIP(hipStreamSynchronize(s));
    }
    if (k == 'F') return std::sqrt(v[0]);
    double r = 0;
    for (double x : v) r = (x != x || x > r) ? x : r;
    return r;
}

}  // namespace native
}  // namespace slate_amd
