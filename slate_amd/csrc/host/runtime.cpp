// Native host runtime: tile-instance coherency table (MOSI), slab memory
// pool bookkeeping, and the trace event recorder.
//
// Parity notes:
//  * TileTable  <-> SLATE TileNode/MatrixStorage coherency
//    (include/slate/internal/MatrixStorage.hh:35-143, 862-1005,
//     include/slate/BaseMatrix.hh:1719-1740, 2640-2720, 3159-3247;
//     SURVEY Appendix A).  One process drives one MI355X, so a tile has at
//    most two instances: slot 0 = host, slot 1 = this rank's device.
//  * SlabPool   <-> SLATE Memory (src/core/Memory.cc:17-220): fixed-size
//    blocks handed out from large chunks (one allocation per chunk, sized
//    for 288 GB HBM), free lists per block size; the Python side maps chunk
//    ids to device/host buffers.
//  * TraceRecorder <-> SLATE trace::Trace (src/auxiliary/Trace.cc): events
//    {name, start, stop, stream/thread, nest} with thread-safe append.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace slate_host {

enum : int { Invalid = 0x001, Shared = 0x010, Modified = 0x100, OnHold = 0x1000 };
static constexpr int NSLOT = 2;  // 0 = host, 1 = device

struct Instance {
    bool exists = false;
    int state = Invalid;   // Invalid / Shared / Modified
    bool hold = false;
    int kind = 0;          // 0 workspace, 1 slate-owned, 2 user-owned
    char layout = 'C';
};

struct Node {
    Instance inst[NSLOT];
    int origin = -1;         // slot of the origin instance (-1: remote tile)
    int64_t receive_count = 0;
};

class TileTable {
public:
    TileTable() = default;

    // Insert / replace an instance. Workspace instances start Invalid,
    // others Shared (MatrixStorage.hh:1107-1109).
    void insert(int64_t i, int64_t j, int slot, int kind, bool origin) {
        std::lock_guard<std::mutex> g(mu_);
        Node& n = nodes_[key(i, j)];
        check_slot(slot);
        Instance& in = n.inst[slot];
        in.exists = true;
        in.kind = kind;
        in.state = (kind == 0) ? Invalid : Shared;
        in.hold = false;
        if (origin) n.origin = slot;
    }
    bool exists(int64_t i, int64_t j, int slot) const {
        std::lock_guard<std::mutex> g(mu_);
        auto it = nodes_.find(key(i, j));
        if (it == nodes_.end()) return false;
        if (slot < 0) {
            for (auto& x : it->second.inst) if (x.exists) return true;
            return false;
        }
        check_slot(slot);
        return it->second.inst[slot].exists;
    }
    int state(int64_t i, int64_t j, int slot) const {
        std::lock_guard<std::mutex> g(mu_);
        const Instance& in = get(i, j, slot);
        return in.state | (in.hold ? OnHold : 0);
    }
    int origin(int64_t i, int64_t j) const {
        std::lock_guard<std::mutex> g(mu_);
        auto it = nodes_.find(key(i, j));
        return it == nodes_.end() ? -1 : it->second.origin;
    }
    // Prepare an acquire of (i,j) on dst.  Returns the slot to copy from,
    // or -1 when dst already holds valid data.  Performs the state
    // transitions of BaseMatrix::tileGet: both ends Shared; with modify,
    // dst Modified and every other instance Invalid; with hold, OnHold.
    int acquire(int64_t i, int64_t j, int dst, bool modify, bool hold) {
        std::lock_guard<std::mutex> g(mu_);
        Node& n = node(i, j);
        check_slot(dst);
        Instance& d = n.inst[dst];
        int src = -1;
        if (!d.exists || d.state == Invalid) {
            // pick a valid source, scanning devices before the host
            for (int s = NSLOT - 1; s >= 0; --s) {
                if (s != dst && n.inst[s].exists && n.inst[s].state != Invalid) { src = s; break; }
            }
            if (src < 0 && d.exists && d.state == Invalid) {
                // no valid copy anywhere: treat dst's content as the truth
                // (e.g. freshly inserted workspace about to be overwritten)
            } else if (src < 0) {
                throw std::runtime_error("tile (" + std::to_string(i) + "," + std::to_string(j) +
                                         ") has no valid instance");
            }
            if (!d.exists) { d.exists = true; d.kind = 0; }
            if (src >= 0) {
                d.state = Shared;
                if (n.inst[src].state == Modified) n.inst[src].state = Shared;
            } else {
                d.state = Shared;
            }
        }
        if (modify) {
            for (int s = 0; s < NSLOT; ++s)
                if (s != dst && n.inst[s].exists) n.inst[s].state = Invalid;
            d.state = Modified;
        }
        if (hold) d.hold = true;
        return src;
    }
    // tileModified (BaseMatrix.hh:1719-1740)
    void modified(int64_t i, int64_t j, int slot, bool permissive) {
        std::lock_guard<std::mutex> g(mu_);
        Node& n = node(i, j);
        check_slot(slot);
        if (!n.inst[slot].exists) throw std::runtime_error("tileModified: missing instance");
        if (!permissive)
            for (int s = 0; s < NSLOT; ++s)
                if (s != slot && n.inst[s].exists && n.inst[s].state == Modified)
                    throw std::runtime_error("tileModified: another instance is Modified");
        for (int s = 0; s < NSLOT; ++s)
            if (s != slot && n.inst[s].exists) n.inst[s].state = Invalid;
        n.inst[slot].state = Modified;
    }
    void set_state(int64_t i, int64_t j, int slot, int st) {
        std::lock_guard<std::mutex> g(mu_);
        Instance& in = node(i, j).inst[slot];
        in.state = st & 0x111;
        in.hold = (st & OnHold) != 0;
    }
    void unhold(int64_t i, int64_t j, int slot) {
        std::lock_guard<std::mutex> g(mu_);
        node(i, j).inst[slot].hold = false;
    }
    // Release a workspace instance if it is neither OnHold nor the last
    // valid copy of a local tile (MatrixStorage.hh:894-933).
    // Returns true when the instance was erased (caller frees the buffer).
    bool release(int64_t i, int64_t j, int slot) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = nodes_.find(key(i, j));
        if (it == nodes_.end()) return false;
        Node& n = it->second;
        Instance& in = n.inst[slot];
        if (!in.exists || in.kind != 0 || in.hold) return false;
        if (n.origin >= 0 && in.state != Invalid) {
            bool other_valid = false;
            for (int s = 0; s < NSLOT; ++s)
                if (s != slot && n.inst[s].exists && n.inst[s].state != Invalid) other_valid = true;
            if (!other_valid) return false;
        }
        in = Instance();
        bool any = false;
        for (auto& x : n.inst) any |= x.exists;
        if (!any) nodes_.erase(it);
        return true;
    }
    void erase(int64_t i, int64_t j, int slot) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = nodes_.find(key(i, j));
        if (it == nodes_.end()) return;
        if (slot < 0) { nodes_.erase(it); return; }
        it->second.inst[slot] = Instance();
        bool any = false;
        for (auto& x : it->second.inst) any |= x.exists;
        if (!any) nodes_.erase(it);
    }
    // Slot holding the latest data (for origin update): -1 if origin valid.
    int update_origin_source(int64_t i, int64_t j) {
        std::lock_guard<std::mutex> g(mu_);
        Node& n = node(i, j);
        if (n.origin < 0) return -1;
        if (n.inst[n.origin].state != Invalid) return -1;
        for (int s = 0; s < NSLOT; ++s)
            if (n.inst[s].exists && n.inst[s].state != Invalid) {
                n.inst[n.origin].state = Shared;
                if (n.inst[s].state == Modified) n.inst[s].state = Shared;
                return s;
            }
        throw std::runtime_error("tileUpdateOrigin: no valid instance");
    }
    int64_t receive_count(int64_t i, int64_t j) const {
        std::lock_guard<std::mutex> g(mu_);
        auto it = nodes_.find(key(i, j));
        return it == nodes_.end() ? 0 : it->second.receive_count;
    }
    int64_t add_receive_count(int64_t i, int64_t j, int64_t d) {
        std::lock_guard<std::mutex> g(mu_);
        Node& n = nodes_[key(i, j)];
        n.receive_count += d;
        if (n.receive_count < 0) n.receive_count = 0;
        return n.receive_count;
    }
    // Bulk: mark every instance in a slot with a state (after a whole-buffer
    // kernel or copy).  Returns number of tiles touched.
    int64_t mark_all(int slot, int st) {
        std::lock_guard<std::mutex> g(mu_);
        int64_t c = 0;
        for (auto& kv : nodes_) {
            Node& n = kv.second;
            if (!n.inst[slot].exists) continue;
            ++c;
            if (st == Modified)
                for (int s = 0; s < NSLOT; ++s)
                    if (s != slot && n.inst[s].exists) n.inst[s].state = Invalid;
            n.inst[slot].state = st;
        }
        return c;
    }
    std::vector<std::tuple<int64_t, int64_t, int>> instances() const {
        std::lock_guard<std::mutex> g(mu_);
        std::vector<std::tuple<int64_t, int64_t, int>> out;
        for (auto& kv : nodes_)
            for (int s = 0; s < NSLOT; ++s)
                if (kv.second.inst[s].exists)
                    out.emplace_back(kv.first.first, kv.first.second, s);
        return out;
    }
    size_t size() const { std::lock_guard<std::mutex> g(mu_); return nodes_.size(); }
    void clear_workspace() {
        std::lock_guard<std::mutex> g(mu_);
        for (auto it = nodes_.begin(); it != nodes_.end();) {
            Node& n = it->second;
            bool any = false;
            for (auto& x : n.inst) {
                if (x.exists && x.kind == 0 && !x.hold && n.origin < 0) x = Instance();
                any |= x.exists;
            }
            if (!any) it = nodes_.erase(it); else ++it;
        }
    }

private:
    struct PairHash {
        size_t operator()(const std::pair<int64_t, int64_t>& p) const {
            return std::hash<int64_t>()(p.first * 1000003 ^ p.second);
        }
    };
    static std::pair<int64_t, int64_t> key(int64_t i, int64_t j) { return {i, j}; }
    static void check_slot(int s) {
        if (s < 0 || s >= NSLOT) throw std::out_of_range("bad memory slot");
    }
    Node& node(int64_t i, int64_t j) {
        auto it = nodes_.find(key(i, j));
        if (it == nodes_.end())
            throw std::out_of_range("tile (" + std::to_string(i) + "," + std::to_string(j) + ") not in table");
        return it->second;
    }
    const Instance& get(int64_t i, int64_t j, int slot) const {
        auto it = nodes_.find(key(i, j));
        if (it == nodes_.end())
            throw std::out_of_range("tile (" + std::to_string(i) + "," + std::to_string(j) + ") not in table");
        check_slot(slot);
        return it->second.inst[slot];
    }
    mutable std::mutex mu_;
    std::unordered_map<std::pair<int64_t, int64_t>, Node, PairHash> nodes_;
};

// Fixed-size block pool: blocks of `block_bytes` carved out of chunks of
// `blocks_per_chunk` blocks.  The Python side allocates one buffer per chunk
// (grow() returns the new chunk id) and maps (chunk, index) to a view.
class SlabPool {
public:
    SlabPool(int64_t block_bytes, int64_t blocks_per_chunk)
        : block_bytes_(block_bytes), per_chunk_(blocks_per_chunk) {
        if (block_bytes <= 0 || blocks_per_chunk <= 0) throw std::invalid_argument("SlabPool sizes");
    }
    // Returns (chunk, index, needs_new_chunk).  When needs_new_chunk is
    // true the caller must allocate chunk `chunk` before using the block.
    std::tuple<int64_t, int64_t, bool> alloc() {
        std::lock_guard<std::mutex> g(mu_);
        bool grew = false;
        if (free_.empty()) {
            int64_t c = nchunks_++;
            for (int64_t b = per_chunk_ - 1; b >= 0; --b) free_.push_back({c, b});
            grew = true;
        }
        auto blk = free_.back();
        free_.pop_back();
        ++in_use_;
        peak_ = std::max(peak_, in_use_);
        return {blk.first, blk.second, grew};
    }
    void free(int64_t chunk, int64_t idx) {
        std::lock_guard<std::mutex> g(mu_);
        if (chunk < 0 || chunk >= nchunks_ || idx < 0 || idx >= per_chunk_)
            throw std::out_of_range("SlabPool.free: bad block");
        free_.push_back({chunk, idx});
        --in_use_;
    }
    int64_t in_use() const { std::lock_guard<std::mutex> g(mu_); return in_use_; }
    int64_t capacity() const { std::lock_guard<std::mutex> g(mu_); return nchunks_ * per_chunk_; }
    int64_t peak() const { std::lock_guard<std::mutex> g(mu_); return peak_; }
    int64_t chunks() const { std::lock_guard<std::mutex> g(mu_); return nchunks_; }
    int64_t block_bytes() const { return block_bytes_; }
    int64_t blocks_per_chunk() const { return per_chunk_; }

private:
    int64_t block_bytes_, per_chunk_;
    int64_t nchunks_ = 0, in_use_ = 0, peak_ = 0;
    std::vector<std::pair<int64_t, int64_t>> free_;
    mutable std::mutex mu_;
};

// Thread-safe trace event recorder (host spans + device spans resolved by
// the Python side from hipEvents).
class TraceRecorder {
public:
    struct Event { std::string name; double start, stop; int64_t lane; int nest; };
    void on() { on_ = true; t0_ = now(); }
    void off() { on_ = false; }
    bool is_on() const { return on_; }
    static double now() {
        using namespace std::chrono;
        return duration<double>(steady_clock::now().time_since_epoch()).count();
    }
    double t0() const { return t0_; }
    void add(const std::string& name, double start, double stop, int64_t lane, int nest) {
        if (!on_) return;
        std::lock_guard<std::mutex> g(mu_);
        events_.push_back({name, start, stop, lane, nest});
    }
    int64_t thread_lane() {
        auto id = std::this_thread::get_id();
        std::lock_guard<std::mutex> g(mu_);
        auto it = lanes_.find(id);
        if (it != lanes_.end()) return it->second;
        int64_t l = (int64_t)lanes_.size();
        lanes_[id] = l;
        return l;
    }
    std::vector<std::tuple<std::string, double, double, int64_t, int>> events() const {
        std::lock_guard<std::mutex> g(mu_);
        std::vector<std::tuple<std::string, double, double, int64_t, int>> out;
        out.reserve(events_.size());
        for (auto& e : events_) out.emplace_back(e.name, e.start, e.stop, e.lane, e.nest);
        return out;
    }
    void clear() { std::lock_guard<std::mutex> g(mu_); events_.clear(); }

private:
    std::atomic<bool> on_{false};
    double t0_ = 0;
    mutable std::mutex mu_;
    std::vector<Event> events_;
    std::map<std::thread::id, int64_t> lanes_;
};

void register_runtime(py::module& m) {
    m.attr("MOSI_Invalid") = (int)Invalid;
    m.attr("MOSI_Shared") = (int)Shared;
    m.attr("MOSI_Modified") = (int)Modified;
    m.attr("MOSI_OnHold") = (int)OnHold;
    py::class_<TileTable>(m, "TileTable")
        .def(py::init<>())
        .def("insert", &TileTable::insert)
        .def("exists", &TileTable::exists)
        .def("state", &TileTable::state)
        .def("origin", &TileTable::origin)
        .def("acquire", &TileTable::acquire)
        .def("modified", &TileTable::modified)
        .def("set_state", &TileTable::set_state)
        .def("unhold", &TileTable::unhold)
        .def("release", &TileTable::release)
        .def("erase", &TileTable::erase)
        .def("update_origin_source", &TileTable::update_origin_source)
        .def("receive_count", &TileTable::receive_count)
        .def("add_receive_count", &TileTable::add_receive_count)
        .def("mark_all", &TileTable::mark_all)
        .def("instances", &TileTable::instances)
        .def("clear_workspace", &TileTable::clear_workspace)
        .def("__len__", &TileTable::size);
    py::class_<SlabPool>(m, "SlabPool")
        .def(py::init<int64_t, int64_t>())
        .def("alloc", &SlabPool::alloc)
        .def("free", &SlabPool::free)
        .def("in_use", &SlabPool::in_use)
        .def("capacity", &SlabPool::capacity)
        .def("peak", &SlabPool::peak)
        .def("chunks", &SlabPool::chunks)
        .def("block_bytes", &SlabPool::block_bytes)
        .def("blocks_per_chunk", &SlabPool::blocks_per_chunk);
    py::class_<TraceRecorder>(m, "TraceRecorder")
        .def(py::init<>())
        .def("on", &TraceRecorder::on)
        .def("off", &TraceRecorder::off)
        .def("is_on", &TraceRecorder::is_on)
        .def_static("now", &TraceRecorder::now)
        .def("t0", &TraceRecorder::t0)
        .def("add", &TraceRecorder::add)
        .def("thread_lane", &TraceRecorder::thread_lane)
        .def("events", &TraceRecorder::events)
        .def("clear", &TraceRecorder::clear);
}

}  // namespace slate_host
