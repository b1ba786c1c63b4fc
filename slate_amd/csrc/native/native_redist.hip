// redistribute(A, B): copy a matrix between two 2D block-cyclic layouts of
// the same global shape -- any tile sizes, any p x q grids over the world
// (SLATE redistribute, include/slate/slate.hh:426; src/redistribute.cc moves
// tile by tile with MPI send/recv).
//
// MI355X design: ownership in a block-cyclic layout is SEPARABLE -- the
// owner of element (i, j) is (row owner of i, column owner of j) -- so the
// elements rank s sends to rank d are exactly the Cartesian product
//   R(s, d) x C(s, d),  R = rows owned by s's process row in A and by d's
//   process row in B, C likewise for columns.
// One gather kernel packs that product out of s's local block (host-built
// row / column index lists), ONE batched point-to-point exchange moves every
// peer's block at once (RCCL group / host transport), one scatter kernel per
// peer places them.  Same-rank pieces go gather -> scatter without the
// exchange.  Memory: the send and receive buffers, together at most the
// local block sizes.
#include <algorithm>
#include <vector>

#include "native_rt.hpp"

namespace slate_amd {
namespace native {

namespace {

template <typename W>
__global__ void __launch_bounds__(256)
gather2d_kernel(i64 nr, i64 nc, const W* __restrict__ src, i64 lds, const i64* __restrict__ ridx,
                const i64* __restrict__ cidx, W* __restrict__ dst) {
    const i64 r = (i64)blockIdx.x * 256 + threadIdx.x;
    if (r >= nr) return;
    const i64 sr = ridx[r];
    for (i64 c = blockIdx.y; c < nc; c += gridDim.y) dst[r + c * nr] = src[sr + cidx[c] * lds];
}

template <typename W>
__global__ void __launch_bounds__(256)
scatter2d_kernel(i64 nr, i64 nc, const W* __restrict__ src, const i64* __restrict__ ridx, const i64* __restrict__ cidx,
                 W* __restrict__ dst, i64 ldd) {
    const i64 r = (i64)blockIdx.x * 256 + threadIdx.x;
    if (r >= nr) return;
    const i64 dr = ridx[r];
    for (i64 c = blockIdx.y; c < nc; c += gridDim.y) dst[dr + cidx[c] * ldd] = src[r + c * nr];
}

struct W16 { unsigned long long a, b; };

// dst (nr x nc, ld nr) = src[ridx, cidx] (or the reverse), elements of
// esize bytes moved as whole words
void move2d(bool gather, size_t esize, i64 nr, i64 nc, const void* src, i64 lds, const i64* ridx, const i64* cidx,
            void* dst, i64 ldd, hipStream_t s) {
    if (nr <= 0 || nc <= 0) return;
    dim3 g((unsigned)((nr + 255) / 256), (unsigned)std::min<i64>(nc, 2048));
    auto go = [&](auto w) {
        using W = decltype(w);
        if (gather)
            hipLaunchKernelGGL(gather2d_kernel<W>, g, dim3(256), 0, s, nr, nc, static_cast<const W*>(src), lds, ridx,
                               cidx, static_cast<W*>(dst));
        else
            hipLaunchKernelGGL(scatter2d_kernel<W>, g, dim3(256), 0, s, nr, nc, static_cast<const W*>(src), ridx, cidx,
                               static_cast<W*>(dst), ldd);
    };
    if (esize == 4) go(0u);
    else if (esize == 8) go(0ull);
    else go(W16{});
    NHIP(hipGetLastError());
}

struct Layout {
    i64 nb;
    int p, q;
    bool in;          // this rank holds a block of the layout
};

// row (or column) indices split by (owner in A, owner in B): for the pair
// (a, b) the global indices owned by process row a of A and row b of B
std::vector<std::vector<std::vector<i64>>> buckets(i64 n, i64 nba, int pa, i64 nbb, int pb) {
    std::vector<std::vector<std::vector<i64>>> out((size_t)pa, std::vector<std::vector<i64>>((size_t)pb));
    for (i64 i = 0; i < n; ++i) out[(size_t)((i / nba) % pa)][(size_t)((i / nbb) % pb)].push_back(i);
    return out;
}

inline i64 g2l(i64 g, i64 nb, int p) { return (g / nb / p) * nb + g % nb; }

}  // namespace

template <typename T>
void redistribute(const Matrix<T>& A, Matrix<T>& B) {
    NTRACE("redistribute", nullptr);
    const Storage& SA = *A.storage();
    Storage& SB = *B.storage();
    if (SA.m != SB.m || SA.n != SB.n) throw Error("native redistribute: A and B must have the same dimensions");
    Runtime& R = rt();
    hipStream_t s = R.main;
    NHIP(hipStreamSynchronize(s));
    const i64 m = SA.m, n = SA.n;
    if (m == 0 || n == 0) return;
    const int P = R.size;
    if (SA.p * SA.q > P || SB.p * SB.q > P) throw Error("native redistribute: grid larger than the world");
    // world rank r <-> (r % p, r / p) (column-major grids, as every native driver)
    auto coords = [](int r, int p) { return std::make_pair(r % p, r / p); };
    const bool inA = R.rank < SA.p * SA.q, inB = R.rank < SB.p * SB.q;
    const auto rb = buckets(m, SA.nb, SA.p, SB.nb, SB.p);
    const auto cb = buckets(n, SA.nb, SA.q, SB.nb, SB.q);
    std::vector<std::unique_ptr<Scratch>> keep;
    auto up = [&](const std::vector<i64>& v) {
        keep.push_back(std::make_unique<Scratch>(std::max<size_t>(v.size(), 1) * sizeof(i64), s));
        if (!v.empty()) upload(keep.back()->p, v.data(), v.size() * sizeof(i64), s);
        return keep.back()->template as<i64>();
    };
    auto local_of = [](const std::vector<i64>& g, i64 nb, int p) {
        std::vector<i64> l(g.size());
        for (size_t k = 0; k < g.size(); ++k) l[k] = g2l(g[k], nb, p);
        return l;
    };
    const size_t es = sizeof(T);
    std::vector<P2P> ops;
    struct Recv { Scratch* buf; const std::vector<i64>* rows; const std::vector<i64>* cols; };
    std::vector<Recv> recvs;
    // sends (and the same-rank piece)
    if (inA) {
        const auto [par, pac] = coords(R.rank, SA.p);
        for (int d = 0; d < SB.p * SB.q; ++d) {
            const auto [pbr, pbc] = coords(d, SB.p);
            const auto& rows = rb[(size_t)par][(size_t)pbr];
            const auto& cols = cb[(size_t)pac][(size_t)pbc];
            if (rows.empty() || cols.empty()) continue;
            const i64 nr = (i64)rows.size(), nc = (i64)cols.size();
            keep.push_back(std::make_unique<Scratch>((size_t)nr * nc * es, s));
            Scratch* buf = keep.back().get();
            move2d(true, es, nr, nc, SA.buf, SA.lld, up(local_of(rows, SA.nb, SA.p)), up(local_of(cols, SA.nb, SA.q)),
                   buf->p, nr, s);
            if (d == R.rank) {
                move2d(false, es, nr, nc, buf->p, nr, up(local_of(rows, SB.nb, SB.p)),
                       up(local_of(cols, SB.nb, SB.q)), SB.buf, SB.lld, s);
            } else {
                ops.push_back({true, d, buf->p, (size_t)nr * nc * es});
            }
        }
    }
    // receives
    if (inB) {
        const auto [pbr, pbc] = coords(R.rank, SB.p);
        for (int src = 0; src < SA.p * SA.q; ++src) {
            if (src == R.rank) continue;
            const auto [par, pac] = coords(src, SA.p);
            const auto& rows = rb[(size_t)par][(size_t)pbr];
            const auto& cols = cb[(size_t)pac][(size_t)pbc];
            if (rows.empty() || cols.empty()) continue;
            keep.push_back(std::make_unique<Scratch>(rows.size() * cols.size() * es, s));
            ops.push_back({false, src, keep.back()->p, rows.size() * cols.size() * es});
            recvs.push_back({keep.back().get(), &rows, &cols});
        }
    }
    if (!ops.empty()) {
        if (!world_comm()) throw Error("native redistribute: no communicator");
        world_comm()->exchange(ops, s);
    }
    for (auto& rv : recvs)
        move2d(false, es, (i64)rv.rows->size(), (i64)rv.cols->size(), rv.buf->p, (i64)rv.rows->size(),
               up(local_of(*rv.rows, SB.nb, SB.p)), up(local_of(*rv.cols, SB.nb, SB.q)), SB.buf, SB.lld, s);
    NHIP(hipStreamSynchronize(s));
}

#define SLATE_NATIVE_REDIST_INST(T) template void redistribute<T>(const Matrix<T>&, Matrix<T>&);
SLATE_NATIVE_REDIST_INST(float)
SLATE_NATIVE_REDIST_INST(double)
SLATE_NATIVE_REDIST_INST(std::complex<float>)
SLATE_NATIVE_REDIST_INST(std::complex<double>)

}  // namespace native
}  // namespace slate_amd
