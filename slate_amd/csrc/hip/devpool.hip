// Per-device, stream-ordered slab pool for workspace tiles.
//
// Role of SLATE's Memory class (src/core/Memory.cc:17-220: per-device stacks
// of fixed-size nb x nb blocks, grown in chunks, freed at clear), redesigned
// for one process per MI355X with HIP streams instead of OpenMP tasks:
//
//  * memory comes from hipMalloc'd chunks (not the torch caching allocator),
//    sized against the device's HBM: the pool never grows beyond
//    `max_bytes` (default: a fraction of the HBM free at creation), so a
//    288 GB part can hold whole trailing matrices of workspace while a
//    runaway loop fails loudly instead of evicting the matrix itself;
//  * free(block, stream) is stream-ordered: it records an event on the
//    freeing stream; the block is handed out again immediately to the same
//    stream (stream order makes that safe), to another stream once the event
//    has completed, or -- when the pool is at its cap -- to another stream
//    after a device-side hipStreamWaitEvent (no host synchronisation);
//  * chunks are exported to PyTorch as DLPack capsules (zero copy); tile
//    views are slices of a chunk tensor.  A chunk is returned to HIP by
//    trim() only when no block of it is in use and no exported view of it is
//    alive.
#include <deque>
#include <iterator>
#include <memory>
#include <mutex>
#include <vector>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include "common.hpp"

namespace py = pybind11;

namespace {

// DLPack (v0.8 ABI, the "dltensor" capsule torch.utils.dlpack consumes)
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
    void* data; DLDevice device; int32_t ndim; DLDataType dtype;
    int64_t* shape; int64_t* strides; uint64_t byte_offset;
};
struct DLManagedTensor {
    DLTensor dl_tensor; void* manager_ctx; void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;
constexpr uint8_t kDLUInt = 1;

struct Chunk {
    void* base = nullptr;
    int views = 0;      // live exported DLPack tensors
    int used = 0;       // blocks handed out
};

struct FreeBlock {
    int chunk, idx;
    hipStream_t stream;     // stream of the last free (nullptr: never used)
    hipEvent_t ev;          // completes when that stream is past the last use
};

struct PoolState {
    std::mutex mu;
    int device;
    size_t block_bytes;
    int blocks_per_chunk;
    size_t max_bytes;
    std::vector<Chunk> chunks;
    std::deque<FreeBlock> freelist;
    std::vector<hipEvent_t> spare_events;
    int64_t in_use = 0, peak = 0, waits = 0, reuse_same = 0, reuse_done = 0;

    ~PoolState() {
        int old = 0;
        if (hipGetDevice(&old) != hipSuccess) return;
        (void)hipSetDevice(device);
        (void)hipDeviceSynchronize();
        for (auto& f : freelist) if (f.ev) (void)hipEventDestroy(f.ev);
        for (auto e : spare_events) (void)hipEventDestroy(e);
        for (auto& c : chunks) if (c.base) (void)hipFree(c.base);
        (void)hipSetDevice(old);
    }
    hipEvent_t take_event() {
        if (!spare_events.empty()) { auto e = spare_events.back(); spare_events.pop_back(); return e; }
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        return e;
    }
    void give_event(hipEvent_t e) { if (e) spare_events.push_back(e); }
};

struct ViewCtx {
    std::shared_ptr<PoolState> st;
    int chunk;
    int64_t shape[1];
    int64_t strides[1];
};

void view_deleter(DLManagedTensor* t) {
    auto* ctx = static_cast<ViewCtx*>(t->manager_ctx);
    {
        std::lock_guard<std::mutex> g(ctx->st->mu);
        ctx->st->chunks[ctx->chunk].views--;
    }
    delete ctx;
    delete t;
}

void capsule_destructor(PyObject* cap) {
    // consumed capsules are renamed "used_dltensor" by the consumer
    if (PyCapsule_IsValid(cap, "dltensor")) {
        auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
        if (t && t->deleter) t->deleter(t);
    }
}

class DevicePool {
public:
    DevicePool(int device, size_t block_bytes, int blocks_per_chunk, size_t max_bytes)
        : st_(std::make_shared<PoolState>()) {
        if (block_bytes == 0 || blocks_per_chunk <= 0) throw std::invalid_argument("DevicePool sizes");
        st_->device = device;
        st_->block_bytes = (block_bytes + 255) / 256 * 256;     // 256-byte aligned blocks
        st_->blocks_per_chunk = blocks_per_chunk;
        if (max_bytes == 0) {
            // HBM sizing policy: at most half of what is free right now
            size_t fr = 0, tot = 0;
            int old = 0;
            HIP_CHECK(hipGetDevice(&old));
            HIP_CHECK(hipSetDevice(device));
            HIP_CHECK(hipMemGetInfo(&fr, &tot));
            HIP_CHECK(hipSetDevice(old));
            max_bytes = fr / 2;
        }
        st_->max_bytes = max_bytes;
    }

    // -> (chunk, idx, byte offset in chunk, grew)
    py::tuple alloc(uintptr_t stream_u) {
        auto* s = st_.get();
        hipStream_t stream = reinterpret_cast<hipStream_t>(stream_u);
        std::lock_guard<std::mutex> g(s->mu);
        // 1) the block most recently freed on this stream (stream order makes
        //    it safe; likely still in L2), 2) a never-used block, 3) one whose
        //    free event has completed
        for (auto it = s->freelist.rbegin(); it != s->freelist.rend(); ++it) {
            if (it->ev == nullptr || it->stream != stream) continue;
            FreeBlock f = *it;
            s->freelist.erase(std::next(it).base());
            s->reuse_same++;
            return hand_out(f, false);
        }
        for (int pass = 0; pass < 2; ++pass) {
            for (auto it = s->freelist.begin(); it != s->freelist.end(); ++it) {
                bool ok = pass == 0 ? it->ev == nullptr : hipEventQuery(it->ev) == hipSuccess;
                if (!ok) continue;
                FreeBlock f = *it;
                s->freelist.erase(it);
                if (pass == 1) s->reuse_done++;
                return hand_out(f, false);
            }
        }
        // 4) grow while under the HBM cap
        size_t chunk_bytes = s->block_bytes * (size_t)s->blocks_per_chunk;
        const bool under_cap = (s->chunks.size() + 1) * chunk_bytes <= s->max_bytes;
        if (!under_cap && s->freelist.empty())
            throw std::runtime_error("DevicePool: HBM cap reached (" + std::to_string(s->max_bytes) +
                                     " bytes) with every block in use");
        if (under_cap) {
            Chunk c;
            int old = 0;
            HIP_CHECK(hipGetDevice(&old));
            HIP_CHECK(hipSetDevice(s->device));
            hipError_t e = hipMalloc(&c.base, chunk_bytes);
            HIP_CHECK(hipSetDevice(old));
            HIP_CHECK(e);
            int ci = (int)s->chunks.size();
            s->chunks.push_back(c);
            for (int i = s->blocks_per_chunk - 1; i >= 1; --i)
                s->freelist.push_back(FreeBlock{ci, i, nullptr, nullptr});
            return hand_out(FreeBlock{ci, 0, nullptr, nullptr}, true);
        }
        // 5) at the cap: take the oldest pending block, ordered behind its
        //    free on the device (no host wait)
        FreeBlock f = s->freelist.front();
        s->freelist.pop_front();
        HIP_CHECK(hipStreamWaitEvent(stream, f.ev, 0));
        s->waits++;
        return hand_out(f, false);
    }

    void free(int chunk, int idx, uintptr_t stream_u) {
        auto* s = st_.get();
        hipStream_t stream = reinterpret_cast<hipStream_t>(stream_u);
        std::lock_guard<std::mutex> g(s->mu);
        if (chunk < 0 || chunk >= (int)s->chunks.size() || idx < 0 || idx >= s->blocks_per_chunk)
            throw std::out_of_range("DevicePool.free: bad block");
        hipEvent_t ev = s->take_event();
        HIP_CHECK(hipEventRecord(ev, stream));
        s->chunks[chunk].used--;
        s->in_use--;
        s->freelist.push_back(FreeBlock{chunk, idx, stream, ev});
    }

    // whole chunk as a flat uint8 DLPack tensor (zero copy)
    py::object chunk_view(int chunk) {
        auto* s = st_.get();
        std::lock_guard<std::mutex> g(s->mu);
        if (chunk < 0 || chunk >= (int)s->chunks.size()) throw std::out_of_range("chunk_view");
        auto* ctx = new ViewCtx{st_, chunk, {(int64_t)(s->block_bytes * s->blocks_per_chunk)}, {1}};
        auto* t = new DLManagedTensor{};
        t->dl_tensor.data = s->chunks[chunk].base;
        t->dl_tensor.device = DLDevice{kDLROCM, s->device};
        t->dl_tensor.ndim = 1;
        t->dl_tensor.dtype = DLDataType{kDLUInt, 8, 1};
        t->dl_tensor.shape = ctx->shape;
        t->dl_tensor.strides = ctx->strides;
        t->dl_tensor.byte_offset = 0;
        t->manager_ctx = ctx;
        t->deleter = view_deleter;
        s->chunks[chunk].views++;
        PyObject* cap = PyCapsule_New(t, "dltensor", capsule_destructor);
        if (!cap) { s->chunks[chunk].views--; delete ctx; delete t; throw py::error_already_set(); }
        return py::reinterpret_steal<py::object>(cap);
    }

    // return fully idle chunks (no block in use, no live view) to HIP; trailing
    // chunks only, so chunk ids stay stable.  Synchronises the device.
    int trim() {
        auto* s = st_.get();
        std::lock_guard<std::mutex> g(s->mu);
        int old = 0;
        HIP_CHECK(hipGetDevice(&old));
        HIP_CHECK(hipSetDevice(s->device));
        HIP_CHECK(hipDeviceSynchronize());
        int freed = 0;
        while (!s->chunks.empty() && s->chunks.back().used == 0 && s->chunks.back().views == 0) {
            int ci = (int)s->chunks.size() - 1;
            for (auto it = s->freelist.begin(); it != s->freelist.end();) {
                if (it->chunk == ci) { s->give_event(it->ev); it = s->freelist.erase(it); }
                else ++it;
            }
            HIP_CHECK(hipFree(s->chunks.back().base));
            s->chunks.pop_back();
            ++freed;
        }
        HIP_CHECK(hipSetDevice(old));
        return freed;
    }

    py::dict stats() {
        auto* s = st_.get();
        std::lock_guard<std::mutex> g(s->mu);
        py::dict d;
        d["in_use"] = s->in_use;
        d["peak"] = s->peak;
        d["chunks"] = (int64_t)s->chunks.size();
        d["capacity"] = (int64_t)s->chunks.size() * s->blocks_per_chunk;
        d["block_bytes"] = (int64_t)s->block_bytes;
        d["blocks_per_chunk"] = s->blocks_per_chunk;
        d["max_bytes"] = (int64_t)s->max_bytes;
        d["device_waits"] = s->waits;
        d["reuse_same_stream"] = s->reuse_same;
        d["reuse_completed"] = s->reuse_done;
        return d;
    }
    size_t block_bytes() const { return st_->block_bytes; }
    int blocks_per_chunk() const { return st_->blocks_per_chunk; }

private:
    py::tuple hand_out(const FreeBlock& f, bool grew) {
        auto* s = st_.get();
        s->give_event(f.ev);
        s->chunks[f.chunk].used++;
        s->in_use++;
        if (s->in_use > s->peak) s->peak = s->in_use;
        return py::make_tuple(f.chunk, f.idx, (int64_t)(f.idx * s->block_bytes), grew);
    }
    std::shared_ptr<PoolState> st_;
};

}  // namespace

void register_devpool(py::module& m) {
    py::class_<DevicePool>(m, "DevicePool")
        .def(py::init<int, size_t, int, size_t>(), py::arg("device"), py::arg("block_bytes"),
             py::arg("blocks_per_chunk"), py::arg("max_bytes") = 0)
        .def("alloc", &DevicePool::alloc, py::arg("stream"))
        .def("free", &DevicePool::free, py::arg("chunk"), py::arg("idx"), py::arg("stream"))
        .def("chunk_view", &DevicePool::chunk_view)
        .def("trim", &DevicePool::trim)
        .def("stats", &DevicePool::stats)
        .def("block_bytes", &DevicePool::block_bytes)
        .def("blocks_per_chunk", &DevicePool::blocks_per_chunk);
}
