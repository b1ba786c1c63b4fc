// Communicator transports of the native runtime (native_rt.hpp):
//   RcclComm -- RCCL over xGMI, stream-ordered, device buffers (production);
//   HostComm -- host-staged TCP full mesh: lets several ranks share one GPU
//               (RCCL refuses two ranks per device), so every p x q path of
//               the native drivers runs on a one-GPU box.
// SLATE_AMD_NATIVE_TRANSPORT selects (default rccl).  Reference: SLATE's
// MPI layer (include/slate/internal/mpi.hh, BaseMatrix.hh:1762-2452), where
// the transport is whatever MPI provides.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <rccl/rccl.h>

#include "native_rt.hpp"

namespace slate_amd {
namespace native {

#define NCCL(x)                                                                                          \
    do {                                                                                                 \
        ncclResult_t r_ = (x);                                                                           \
        if (r_ != ncclSuccess) throw Error(std::string("RCCL: ") + ncclGetErrorString(r_) + " at " #x);  \
    } while (0)

static int env_int(const char* k, int def) {
    const char* v = std::getenv(k);
    return v && *v ? std::atoi(v) : def;
}

// ------------------------------------------------------------ sockets
static void send_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
        const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
        if (w <= 0) throw Error("native transport: send failed");
        c += w;
        n -= (size_t)w;
    }
}
static void recv_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
        const ssize_t g = ::recv(fd, c, n, 0);
        if (g <= 0) throw Error("native transport: recv failed (peer gone)");
        c += g;
        n -= (size_t)g;
    }
}
static int connect_retry(const char* addr, int port) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(addr, std::to_string(port).c_str(), &hints, &res) != 0 || !res)
        throw Error(std::string("native transport: cannot resolve ") + addr);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
            int one = 1;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            freeaddrinfo(res);
            return fd;
        }
        close(fd);
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
            throw Error("native transport: no connection to " + std::string(addr) + ":" + std::to_string(port));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}
static int listen_on(int port, int backlog) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    sa.sin_port = htons((uint16_t)port);
    if (bind(fd, (sockaddr*)&sa, sizeof(sa)) != 0 || listen(fd, backlog) != 0)
        throw Error("native transport: cannot listen on port " + std::to_string(port));
    return fd;
}
static int base_port() { return env_int("SLATE_AMD_NATIVE_PORT", env_int("MASTER_PORT", 29500) + 1); }
static const char* master_addr() {
    const char* a = std::getenv("MASTER_ADDR");
    return a ? a : "127.0.0.1";
}

// ------------------------------------------------------------ RCCL
static ncclDataType_t nccl_real(DT d, size_t& count) {
    switch (d) {
        case DT::F32: return ncclFloat32;
        case DT::F64: return ncclFloat64;
        case DT::C32: count *= 2; return ncclFloat32;
        case DT::C64: count *= 2; return ncclFloat64;
        case DT::I64: return ncclInt64;
        default: return ncclUint8;
    }
}

class RcclComm : public Comm {
public:
    ncclComm_t c = nullptr;
    ~RcclComm() override { if (c) ncclCommDestroy(c); }
    void bcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        if (size > 1 && bytes) NCCL(ncclBroadcast(buf, buf, bytes, ncclUint8, root, c, s));
    }
    void allreduce(void* buf, size_t count, DT dt, char op, hipStream_t s) override {
        if (size == 1 || !count) return;
        const ncclDataType_t t = nccl_real(dt, count);
        const ncclRedOp_t o = op == 'M' ? ncclMax : op == 'm' ? ncclMin : ncclSum;
        NCCL(ncclAllReduce(buf, buf, count, t, o, c, s));
    }
    void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        if (size == 1) {
            if (recv != send && bytes) dcopy(recv, send, bytes, s);
            return;
        }
        if (bytes) NCCL(ncclAllGather(send, recv, bytes, ncclUint8, c, s));
    }
    void exchange(const std::vector<P2P>& ops, hipStream_t s) override {
        if (ops.empty()) return;
        NCCL(ncclGroupStart());
        for (const P2P& o : ops) {
            if (!o.bytes) continue;
            if (o.send) NCCL(ncclSend(o.buf, o.bytes, ncclUint8, o.peer, c, s));
            else NCCL(ncclRecv(o.buf, o.bytes, ncclUint8, o.peer, c, s));
        }
        NCCL(ncclGroupEnd());
    }
    std::unique_ptr<Comm> split(int colour, int key) override {
        auto out = std::make_unique<RcclComm>();
        NCCL(ncclCommSplit(c, colour, key, &out->c, nullptr));
        int n = 0, r = 0;
        NCCL(ncclCommCount(out->c, &n));
        NCCL(ncclCommUserRank(out->c, &r));
        out->size = n;
        out->rank = r;
        // world ranks of the members: one all-gather over the new comm
        out->world.assign((size_t)n, 0);
        int* d = nullptr;
        NHIP(hipMalloc(&d, sizeof(int) * n));
        int me = world[rank];
        upload(d + r, &me, sizeof(int), rt().main);
        NCCL(ncclAllGather(d + r, d, 1, ncclInt32, out->c, rt().main));
        NHIP(hipMemcpyAsync(out->world.data(), d, sizeof(int) * n, hipMemcpyDeviceToHost, rt().main));
        NHIP(hipStreamSynchronize(rt().main));
        NHIP(hipFree(d));
        return out;
    }
};

// rank 0 serves the RCCL unique id on a TCP port; the others connect
static void nccl_bootstrap(ncclUniqueId* id, int rank, int size) {
    const int port = base_port();
    if (rank == 0) {
        NCCL(ncclGetUniqueId(id));
        int fd = listen_on(port, size);
        for (int r = 1; r < size; ++r) {
            int c = accept(fd, nullptr, nullptr);
            if (c < 0) throw Error("native bootstrap: accept failed");
            send_all(c, id, sizeof(*id));
            close(c);
        }
        close(fd);
        return;
    }
    int fd = connect_retry(master_addr(), port);
    recv_all(fd, id, sizeof(*id));
    close(fd);
}

// ------------------------------------------------------------ host TCP
struct Mesh {
    int rank = 0, size = 1;
    std::vector<int> fd;           // socket to each world rank (-1: self)
};
static Mesh& mesh() {
    static Mesh m;
    return m;
}

// every rank listens on base + 1 + rank; rank r connects to every lower rank
// and accepts every higher one (the connector announces its rank)
static void mesh_init(int rank, int size) {
    Mesh& M = mesh();
    M.rank = rank;
    M.size = size;
    M.fd.assign((size_t)size, -1);
    const int port0 = base_port() + 1;
    int lfd = listen_on(port0 + rank, size);
    for (int r = 0; r < rank; ++r) {
        int fd = connect_retry(master_addr(), port0 + r);
        int32_t me = rank;
        send_all(fd, &me, sizeof(me));
        M.fd[r] = fd;
    }
    for (int k = rank + 1; k < size; ++k) {
        int fd = accept(lfd, nullptr, nullptr);
        if (fd < 0) throw Error("native transport: accept failed");
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        int32_t who = -1;
        recv_all(fd, &who, sizeof(who));
        if (who <= rank || who >= size) throw Error("native transport: bad peer id");
        M.fd[who] = fd;
    }
    close(lfd);
}

template <typename R>
static void reduce_into(R* acc, const R* x, size_t n, char op) {
    for (size_t i = 0; i < n; ++i) {
        if (op == 'M') acc[i] = (x[i] != x[i] || x[i] > acc[i]) ? x[i] : acc[i];
        else if (op == 'm') acc[i] = (x[i] != x[i] || x[i] < acc[i]) ? x[i] : acc[i];
        else acc[i] += x[i];
    }
}

class HostComm : public Comm {
public:
    int fd_of(int member) const { return mesh().fd[world[member]]; }
    // copies on the caller's stream, completed before returning (a
    // null-stream hipMemcpy does not order against non-blocking streams and
    // a pageable host->device copy may return before the DMA has landed)
    void d2h(std::vector<char>& h, const void* d, size_t bytes, hipStream_t s) {
        h.resize(bytes);
        if (bytes) NHIP(hipMemcpyAsync(h.data(), d, bytes, hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
    }
    void h2d(void* d, const std::vector<char>& h, size_t bytes, hipStream_t s) {
        if (bytes) upload(d, h.data(), bytes, s);
        NHIP(hipStreamSynchronize(s));
    }
    void bcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        if (size == 1 || !bytes) return;
        std::vector<char> h;
        if (rank == root) {
            d2h(h, buf, bytes, s);
            for (int r = 0; r < size; ++r)
                if (r != root) send_all(fd_of(r), h.data(), bytes);
        } else {
            NHIP(hipStreamSynchronize(s));
            h.resize(bytes);
            recv_all(fd_of(root), h.data(), bytes);
            h2d(buf, h, bytes, s);
        }
    }
    void allreduce(void* buf, size_t count, DT dt, char op, hipStream_t s) override {
        if (size == 1 || !count) return;
        const size_t bytes = count * dt_size(dt);
        std::vector<char> h, t(bytes);
        d2h(h, buf, bytes, s);
        if (rank == 0) {
            for (int r = 1; r < size; ++r) {
                recv_all(fd_of(r), t.data(), bytes);
                switch (dt) {
                    case DT::F32: reduce_into((float*)h.data(), (const float*)t.data(), count, op); break;
                    case DT::C32: reduce_into((float*)h.data(), (const float*)t.data(), 2 * count, op); break;
                    case DT::F64: reduce_into((double*)h.data(), (const double*)t.data(), count, op); break;
                    case DT::C64: reduce_into((double*)h.data(), (const double*)t.data(), 2 * count, op); break;
                    case DT::I64: reduce_into((int64_t*)h.data(), (const int64_t*)t.data(), count, op); break;
                    default: reduce_into((uint8_t*)h.data(), (const uint8_t*)t.data(), bytes, op); break;
                }
            }
            for (int r = 1; r < size; ++r) send_all(fd_of(r), h.data(), bytes);
        } else {
            send_all(fd_of(0), h.data(), bytes);
            recv_all(fd_of(0), h.data(), bytes);
        }
        h2d(buf, h, bytes, s);
    }
    void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        std::vector<char> mine, all((size_t)size * bytes);
        d2h(mine, send, bytes, s);
        if (bytes) std::memcpy(all.data() + (size_t)rank * bytes, mine.data(), bytes);
        // pairwise in ascending peer order: the lower rank sends first
        for (int r = 0; r < size; ++r) {
            if (r == rank || !bytes) continue;
            if (rank < r) {
                send_all(fd_of(r), mine.data(), bytes);
                recv_all(fd_of(r), all.data() + (size_t)r * bytes, bytes);
            } else {
                recv_all(fd_of(r), all.data() + (size_t)r * bytes, bytes);
                send_all(fd_of(r), mine.data(), bytes);
            }
        }
        h2d(recv, all, all.size(), s);
    }
    void exchange(const std::vector<P2P>& ops, hipStream_t s) override {
        NHIP(hipStreamSynchronize(s));
        std::vector<int> peers;
        for (const P2P& o : ops) peers.push_back(o.peer);
        std::sort(peers.begin(), peers.end());
        peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
        for (int r : peers) {
            auto do_sends = [&] {
                for (const P2P& o : ops)
                    if (o.send && o.peer == r && o.bytes) {
                        std::vector<char> h;
                        d2h(h, o.buf, o.bytes, s);
                        send_all(fd_of(r), h.data(), o.bytes);
                    }
            };
            auto do_recvs = [&] {
                for (const P2P& o : ops)
                    if (!o.send && o.peer == r && o.bytes) {
                        std::vector<char> h(o.bytes);
                        recv_all(fd_of(r), h.data(), o.bytes);
                        h2d(o.buf, h, o.bytes, s);
                    }
            };
            if (rank < r) { do_sends(); do_recvs(); }
            else { do_recvs(); do_sends(); }
        }
    }
    std::unique_ptr<Comm> split(int colour, int key) override {
        // every member learns every (colour, key, world rank) triple
        struct CK { int32_t colour, key, world; };
        CK me{colour, key, world[rank]};
        std::vector<CK> all((size_t)size);
        all[rank] = me;
        for (int r = 0; r < size; ++r) {
            if (r == rank) continue;
            if (rank < r) {
                send_all(fd_of(r), &me, sizeof(me));
                recv_all(fd_of(r), &all[r], sizeof(CK));
            } else {
                recv_all(fd_of(r), &all[r], sizeof(CK));
                send_all(fd_of(r), &me, sizeof(me));
            }
        }
        std::vector<CK> sel;
        for (const CK& c : all)
            if (c.colour == colour) sel.push_back(c);
        std::stable_sort(sel.begin(), sel.end(), [](const CK& a, const CK& b) {
            return a.key != b.key ? a.key < b.key : a.world < b.world;
        });
        auto out = std::make_unique<HostComm>();
        out->size = (int)sel.size();
        for (size_t i = 0; i < sel.size(); ++i) {
            out->world.push_back(sel[i].world);
            if (sel[i].world == world[rank]) out->rank = (int)i;
        }
        return out;
    }
};

// ------------------------------------------------------------ selection
static std::unique_ptr<Comm> g_world;
static std::string g_name = "none";

void transport_init(int rank, int size) {
    if (size <= 1) return;
    const char* t = std::getenv("SLATE_AMD_NATIVE_TRANSPORT");
    const std::string kind = t ? t : "rccl";
    if (kind == "host") {
        mesh_init(rank, size);
        auto w = std::make_unique<HostComm>();
        w->size = size;
        w->rank = rank;
        for (int r = 0; r < size; ++r) w->world.push_back(r);
        g_world = std::move(w);
        g_name = "host";
    } else {
        ncclUniqueId id;
        nccl_bootstrap(&id, rank, size);
        auto w = std::make_unique<RcclComm>();
        NCCL(ncclCommInitRank(&w->c, size, id, rank));
        w->size = size;
        w->rank = rank;
        for (int r = 0; r < size; ++r) w->world.push_back(r);
        g_world = std::move(w);
        g_name = "rccl";
    }
}

void transport_finalize() {
    g_world.reset();
    Mesh& M = mesh();
    for (int& fd : M.fd)
        if (fd >= 0) { close(fd); fd = -1; }
    g_name = "none";
}

Comm* world_comm() { return g_world.get(); }
const char* transport_name() { return g_name.c_str(); }

}  // namespace native
}  // namespace slate_amd
