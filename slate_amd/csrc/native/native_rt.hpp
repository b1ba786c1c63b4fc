// Internal header of the native (Python-free) runtime: process runtime,
// communicator transports, distributed storage and small helpers shared by
// native.hip (drivers), native_comm.hip (transports) and capi_native.hip
// (C / LAPACK / ScaLAPACK / BLACS ABI).  Not installed.
#pragma once
#include <complex>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include <hip/hip_runtime.h>

#include "../hip/common.hpp"
#include "../hip/devalloc.hpp"
#include "../hip/kernels.hpp"
#include "../hip/launchers.hpp"
#include "slate_amd/slate_native.hh"

namespace slate_amd {
namespace native {

using slate_hip::i64;

#define NHIP(x)                                                                                          \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) throw ::slate_amd::native::Error(std::string("HIP: ") + hipGetErrorString(e_) + " at " #x);     \
    } while (0)

// ------------------------------------------------------------ transports
// A communicator over a subset of the world ranks.  Two implementations:
//   * RCCL (ncclComm_t, ncclCommSplit for sub-communicators): stream-ordered,
//     device buffers, one hop over xGMI -- the production transport;
//   * host-staged TCP (every rank connected to every other at start-up): the
//     stream is synchronised, buffers go device -> host -> socket -> host ->
//     device.  It lets several ranks share ONE GPU (RCCL refuses that), so
//     the p x q drivers run on a one-GPU box (tests) and on machines without
//     RCCL peers.  SLATE_AMD_NATIVE_TRANSPORT = rccl | host.
enum class DT : int { F32 = 0, F64 = 1, C32 = 2, C64 = 3, I64 = 4, U8 = 5 };
inline size_t dt_size(DT d) {
    switch (d) {
        case DT::F32: return 4;
        case DT::F64: return 8;
        case DT::C32: return 8;
        case DT::C64: return 16;
        case DT::I64: return 8;
        default: return 1;
    }
}
template <typename T> struct dt_of;
template <> struct dt_of<float> { static constexpr DT v = DT::F32; };
template <> struct dt_of<double> { static constexpr DT v = DT::F64; };
template <> struct dt_of<std::complex<float>> { static constexpr DT v = DT::C32; };
template <> struct dt_of<std::complex<double>> { static constexpr DT v = DT::C64; };
template <> struct dt_of<int64_t> { static constexpr DT v = DT::I64; };

struct P2P {                       // one point-to-point transfer of a batch
    bool send;
    int peer;                      // rank inside the communicator
    void* buf;                     // device pointer
    size_t bytes;
};

class Comm {
public:
    int size = 1, rank = 0;
    std::vector<int> world;        // world rank of each member
    virtual ~Comm() = default;
    // all stream-ordered from the caller's point of view (the host transport
    // synchronises s first and returns with the result in place)
    virtual void bcast(void* buf, size_t bytes, int root, hipStream_t s) = 0;
    // op: 's' sum, 'M' max, 'm' min (max / min: real types only)
    virtual void allreduce(void* buf, size_t count, DT dt, char op, hipStream_t s) = 0;
    // recv = size blocks of `bytes`, block r from member r
    virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
    virtual void exchange(const std::vector<P2P>& ops, hipStream_t s) = 0;
    // members of this communicator with colour == mine, ordered by key
    virtual std::unique_ptr<Comm> split(int colour, int key) = 0;
};

// the world communicator of the selected transport (nullptr: one rank)
Comm* world_comm();
void transport_init(int rank, int size);
void transport_finalize();
const char* transport_name();

// ------------------------------------------------------------ runtime
// Peer-mapped mailboxes of one communicator (csrc/hip/lu_dist.hip
// lu_dist_base_kernel; Python twin: parallel/peer.py): my uncached mailbox,
// exported by IPC handle, and every peer's mailbox opened in my address
// space.  Created collectively on first use; SLATE_AMD_LU_PEER=0 disables.
struct PeerBox {
    void* own = nullptr;
    std::vector<void*> opened;
    unsigned long long* mbox_d = nullptr;   // device array [size]: mailbox of each member
    char* part = nullptr;                   // intra-rank partial slots
    unsigned long long* err = nullptr;      // timeout word
    long long seq = 0;                      // next sequence base (identical on every member)
    long long launches = 0;
    bool dead = false;                      // a kernel timed out: tags no longer agree, never reuse
    ~PeerBox();
};
PeerBox* peer_box(Comm* c, std::unique_ptr<PeerBox>& slot, hipStream_t s);

struct GridComms {
    int p = 1, q = 1, pr = 0, pc = 0;
    std::unique_ptr<Comm> row;     // same process row, ranked by pc
    std::unique_ptr<Comm> col;     // same process column, ranked by pr
    std::unique_ptr<Comm> colu;    // a second `col` for the update stream (p > 1)
    std::unique_ptr<PeerBox> colpeer;   // mailboxes of the column (distributed LU panel)
};

struct Runtime {
    bool up = false;
    int rank = 0, size = 1, local = 0, device = 0;
    hipStream_t main = nullptr, panel = nullptr, update = nullptr, comm = nullptr;
    int update_res = 0;     // CUs the live update stream leaves free (set_update_reservation)
    std::map<int, hipStream_t> parked;   // update streams of the other reservations (kept, not destroyed)
    void* lu_work = nullptr;
    void* qr_work = nullptr;
    std::map<std::pair<int, int>, std::unique_ptr<GridComms>> grids;
    std::mutex mu;
};
Runtime& rt();
// Re-create the update stream so that it leaves `cus` compute units free of
// its workgroups (0: unmasked).  Drains the old stream first.  The process
// keeps FOUR streams (main, panel, update, comm) -- the box's hardware queues.
void set_update_reservation(int cus);

GridComms* grid_comms(int p, int q);

// ------------------------------------------------------------ storage
struct Storage {
    i64 m = 0, n = 0, nb = 1;
    int p = 1, q = 1, pr = 0, pc = 0;
    i64 mloc = 0, nloc = 0, lld = 1;
    size_t esize = 8;
    void* buf = nullptr;
    bool owns = true;
    std::shared_ptr<Storage> parent;   // a view keeps the storage it points into alive
    GridComms* gc = nullptr;
    ~Storage() {
        if (buf && owns) (void)hipFree(buf);
    }
};

inline i64 numroc(i64 n, i64 nb, int iproc, int nprocs) {
    const i64 nblocks = n / nb;
    i64 num = (nblocks / nprocs) * nb;
    const i64 extra = nblocks % nprocs;
    if (iproc < extra) num += nb;
    else if (iproc == extra) num += n % nb;
    return num;
}
inline i64 l2g(i64 l, i64 nb, int p, int pr) { return ((l / nb) * p + pr) * nb + l % nb; }
inline i64 tiles_before(i64 t, int p, int pr) { return t > pr ? (t - pr + p - 1) / p : 0; }

// kernel element type of an API type
template <typename T> struct kt_of { using type = T; };
template <> struct kt_of<std::complex<float>> { using type = slate_hip::ccplx; };
template <> struct kt_of<std::complex<double>> { using type = slate_hip::zcplx; };
template <typename T> using K = typename kt_of<T>::type;
template <typename T> inline K<T>* kp(T* p) { return reinterpret_cast<K<T>*>(p); }
template <typename T> inline const K<T>* kp(const T* p) { return reinterpret_cast<const K<T>*>(p); }
template <typename T> inline K<T> kv(T v) {
    K<T> r;
    std::memcpy(&r, &v, sizeof(T));
    return r;
}
template <typename T> constexpr bool is_cplx() { return !std::is_same<T, float>::value && !std::is_same<T, double>::value; }
template <typename T> constexpr char ctrans() { return is_cplx<T>() ? 'C' : 'T'; }
// op(view(A)) for a view whose op is `view` (real types: ConjTrans == Trans):
// T T = C C = NoTrans; a conjugation without transposition is not a view
template <typename T> inline Op compose_op(Op outer, Op view) {
    auto canon = [](Op o) { return (!is_cplx<T>() && o == Op::ConjTrans) ? Op::Trans : o; };
    outer = canon(outer);
    view = canon(view);
    if (view == Op::NoTrans) return outer;
    if (outer == Op::NoTrans) return view;
    if (outer == view) return Op::NoTrans;
    throw Error("native: conj(A) (a conjugate without transpose) is not a view");
}
template <typename T> inline T conj_of(T x) {
    if constexpr (is_cplx<T>()) return std::conj(x);
    else return x;
}

// ------------------------------------------------------------ small RAII
struct Event {
    hipEvent_t e = nullptr;
    Event() { NHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming)); }
    ~Event() { if (e) (void)hipEventDestroy(e); }
    Event(const Event&) = delete;
    void record(hipStream_t s) { NHIP(hipEventRecord(e, s)); }
    void wait(hipStream_t s) const { NHIP(hipStreamWaitEvent(s, e, 0)); }
};

// host -> device upload, complete on return, and device -> device copies:
// kernel copies (native_copy.hip) -- never a copy-engine write into device
// memory that kernels on other XCDs may hold in their L2
void upload(void* d, const void* h, size_t bytes, hipStream_t s);
void dcopy(void* d, const void* src, size_t bytes, hipStream_t s);
// zero fill BY KERNEL (stream-ordered): hipMemsetAsync may run on a copy
// engine, whose writes a later kernel does not see while an XCD's L2 still
// holds the buffer's old lines (cached scratch blocks are reused: stale
// progress counters of a bulge chase made it skip its waits)
void dzero(void* d, size_t bytes, hipStream_t s);
// dst[:, didx[c]] = src[:, sidx[c]] for c < ncols (m elements of esize bytes
// per column; host index lists); complete on return
void copy_cols(void* dst, i64 ldd, const i64* didx, const void* src, i64 lds, const i64* sidx, i64 m, size_t esize,
               i64 ncols, hipStream_t s);

// stream b waits for everything issued so far on stream a
inline void join(hipStream_t a, hipStream_t b) {
    Event ev;
    ev.record(a);
    ev.wait(b);
}

// device scratch: cached hipMalloc'd blocks, reuse ordered by events
// (csrc/hip/devalloc.hpp -- not the stream-ordered pool); freed after the
// owning stream reaches the destructor's point
struct Scratch {
    void* p = nullptr;
    hipStream_t s = nullptr;
    Scratch(size_t bytes, hipStream_t st) : s(st) {
        if (!bytes) return;
        p = slate_hip::dev_alloc(bytes, st);
        if (poison()) NHIP(hipMemsetAsync(p, 0xFF, bytes, st));     // NaN: exposes reads before writes (diagnostics)
    }
    // diagnostics: SLATE_AMD_NATIVE_POISON=1 fills every scratch buffer with NaN
    static bool poison() {
        static const bool on = [] { const char* e = std::getenv("SLATE_AMD_NATIVE_POISON"); return e && *e == '1'; }();
        return on;
    }
    // a buffer that outlives finalize() (e.g. QRFactors held by the caller)
    // must not record on its destroyed stream
    ~Scratch() { if (p) slate_hip::dev_free(p, rt().up ? s : nullptr); }
    Scratch(const Scratch&) = delete;
    template <typename T> T* as() { return static_cast<T*>(p); }
};

// ------------------------------------------------------------ kernel helpers
// (shared by the driver files native.hip / native_eig.hip)
template <typename T>
inline void gemm_k(char ta, char tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda, const T* B, i64 ldb, T beta,
            T* C, i64 ldc, hipStream_t s, const slate_hip::TriMask* mask = nullptr) {
    if (m <= 0 || n <= 0) return;
    slate_hip::GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = (double)std::real(alpha); c.alpha_im = (double)std::imag(alpha);
    c.beta_re = (double)std::real(beta); c.beta_im = (double)std::imag(beta);
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    if (mask) c.mask = *mask;
    if constexpr (is_cplx<T>()) slate_hip::gemm_complex<K<T>>(c, s);
    else slate_hip::gemm_real<T>(c, s);
}

// device-to-device block copy: the gecopy kernel (hipMemcpy2DAsync between
// device pitches gave wrong results on this stack for pitched copies of a
// few MB -- tools/probe/native_probe.cc)
template <typename T>
inline void copy2d(T* dst, i64 ldd, const T* src, i64 lds, i64 m, i64 n, hipStream_t s) {
    if (m > 0 && n > 0) slate_hip::gecopy<K<T>, K<T>>('G', 'N', m, n, kp(src), lds, kp(dst), ldd, s);
}

// ------------------------------------------------------------ tracing (native_trace.hip)
namespace trace_rt {
extern bool g_on;
// one traced scope: a host span, and with a stream a device span (timing
// event pair around the work enqueued on it meanwhile); the name must be a
// string literal.  Costs one branch when tracing is off.
class Scope {
public:
    explicit Scope(const char* name, hipStream_t s = nullptr);
    ~Scope();
    Scope(const Scope&) = delete;
    Scope& operator=(const Scope&) = delete;

private:
    const char* name_;
    hipStream_t s_;
    hipEvent_t evb_ = nullptr, eve_ = nullptr;
    double t0_ = -1;
};
void auto_start();     // SLATE_AMD_NATIVE_TRACE=<path> (initialize)
void auto_finish();    // (finalize)
}  // namespace trace_rt
#define NTRACE_CAT2(a, b) a##b
#define NTRACE_CAT(a, b) NTRACE_CAT2(a, b)
#define NTRACE(name, stream) ::slate_amd::native::trace_rt::Scope NTRACE_CAT(ntrace_scope_, __LINE__)(name, stream)

// lower-triangle mask of a local block whose (0, 0) is local (r0, c0) of a
// block-cyclic matrix (the Python drivers' (1, nb, p, pr, q, pc, r0, c0, 0))
inline slate_hip::TriMask lower_mask(i64 nb, int p, int pr, int q, int pc, i64 r0, i64 c0) {
    slate_hip::TriMask t;
    t.mode = 1; t.nb = nb; t.p = p; t.pr = pr; t.q = q; t.pc = pc; t.row_off = r0; t.col_off = c0; t.diag_off = 0;
    return t;
}

// full matrix of a stored triangle (native.hip): kind 0 = triangular (the
// other part zero, a Unit diagonal set to one), 1 = Hermitian, 2 = symmetric
template <typename T>
Matrix<T> expand_tri(const Matrix<T>& A, Uplo uplo, int kind, Diag diag = Diag::NonUnit);

}  // namespace native
}  // namespace slate_amd
