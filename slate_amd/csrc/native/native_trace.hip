// Native tracing and timers (SLATE src/auxiliary/Trace.cc:359-644,
// slate::timers of src/posv.cc:76-93) for the Python-free library.
//
// MI355X design: the drivers are asynchronous (panel / update / comm
// streams, no host synchronisation inside a factorization), so host
// timestamps alone say little.  A traced scope records
//   * a HOST span (steady clock) on the "host" track of its rank, and
//   * a DEVICE span: a timing hipEvent pair around the work it enqueues on
//     its stream, resolved at finish() against a base event recorded on the
//     main stream when tracing started -- one track per stream (main,
//     panel, update, comm), so the lookahead overlap is visible as it ran.
// finish() gathers every rank's events to rank 0 (one all-gather over the
// world communicator) and writes one Chrome trace-event JSON (chrome://
// tracing, Perfetto): pid = rank, tid = track.  Off by default; a scope then
// costs one branch.  SLATE_AMD_NATIVE_TRACE=<path> turns tracing on at
// initialize() and writes <path> at finalize().
//
// timers(): seconds per scope name, host wall time of each traced scope
// (the drivers end in a stream synchronisation, so a driver's top scope is
// its elapsed time) plus, after finish() or timers() resolves them, the
// device time of each device span under "<name>@device".
#include <chrono>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "native_rt.hpp"

namespace slate_amd {
namespace native {

namespace trace_rt {

bool g_on = false;

namespace {

struct DevSpan {
    std::string name;
    int track;
    hipEvent_t b = nullptr, e = nullptr;
};
struct HostSpan {
    std::string name;
    double t0, t1;      // seconds since the trace base
};

std::mutex g_mu;
std::vector<DevSpan> g_dev;
std::vector<HostSpan> g_host;
std::map<std::string, double> g_timers;
hipEvent_t g_base = nullptr;
std::chrono::steady_clock::time_point g_tbase = std::chrono::steady_clock::now();
std::string g_auto_path;

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - g_tbase).count();
}

int track_of(hipStream_t s) {
    Runtime& R = rt();
    if (s == R.panel) return 1;
    if (s == R.update) return 2;
    if (s == R.comm) return 3;
    return 0;
}
const char* track_name(int t) {
    static const char* n[] = {"main stream", "panel stream", "update stream", "comm stream", "host"};
    return n[t];
}

void json_escape(std::string& out, const std::string& s) {
    for (char c : s) {
        if (c == '"' || c == '\\') out += '\\';
        out += c;
    }
}

// device spans -> (name, track, t0, t1) in seconds since base; adds their
// durations to the timers; clears the pending list
struct Resolved {
    std::string name;
    int track;
    double t0, t1;
};
std::vector<Resolved> g_resolved;

void resolve_locked() {
    for (auto& d : g_dev) {
        NHIP(hipEventSynchronize(d.e));
        float a = 0, b = 0;
        NHIP(hipEventElapsedTime(&a, g_base, d.b));
        NHIP(hipEventElapsedTime(&b, g_base, d.e));
        g_resolved.push_back({d.name, d.track, a * 1e-3, b * 1e-3});
        g_timers[d.name + "@device"] += (b - a) * 1e-3;
        (void)hipEventDestroy(d.b);
        (void)hipEventDestroy(d.e);
    }
    g_dev.clear();
}

}  // namespace

Scope::Scope(const char* name, hipStream_t s) : name_(name), s_(s) {
    if (!g_on) return;
    t0_ = now_s();
    if (s_) {
        NHIP(hipEventCreate(&evb_));
        NHIP(hipEventCreate(&eve_));
        NHIP(hipEventRecord(evb_, s_));
    }
}

Scope::~Scope() {
    if (!g_on || t0_ < 0) return;
    const double t1 = now_s();
    std::lock_guard<std::mutex> lk(g_mu);
    if (s_) {
        if (hipEventRecord(eve_, s_) == hipSuccess) g_dev.push_back({name_, track_of(s_), evb_, eve_});
    }
    g_host.push_back({name_, t0_, t1});
    g_timers[name_] += t1 - t0_;
}

void auto_start() {
    const char* p = std::getenv("SLATE_AMD_NATIVE_TRACE");
    if (p && *p && std::string(p) != "0" && std::string(p) != "1") {
        g_auto_path = p;
        trace::on();
    }
}

void auto_finish() {
    if (!g_auto_path.empty() && g_on) {
        const std::string p = g_auto_path;
        g_auto_path.clear();
        trace::finish(p);
    }
}

}  // namespace trace_rt

namespace trace {

void on() {
    initialize();
    std::lock_guard<std::mutex> lk(trace_rt::g_mu);
    if (trace_rt::g_on) return;
    Runtime& R = rt();
    NHIP(hipDeviceSynchronize());
    if (!trace_rt::g_base) NHIP(hipEventCreate(&trace_rt::g_base));
    NHIP(hipEventRecord(trace_rt::g_base, R.main));
    NHIP(hipEventSynchronize(trace_rt::g_base));
    trace_rt::g_tbase = std::chrono::steady_clock::now();
    trace_rt::g_host.clear();
    trace_rt::g_dev.clear();
    trace_rt::g_resolved.clear();
    trace_rt::g_on = true;
}

void off() {
    trace_rt::g_on = false;
}

bool enabled() { return trace_rt::g_on; }

void finish(const std::string& path) {
    Runtime& R = rt();
    std::string mine;
    {
        std::lock_guard<std::mutex> lk(trace_rt::g_mu);
        trace_rt::g_on = false;
        trace_rt::resolve_locked();
        // this rank's events (pid = rank)
        char buf[256];
        auto ev = [&](const std::string& name, int track, double t0, double t1) {
            mine += "{\"name\":\"";
            trace_rt::json_escape(mine, name);
            std::snprintf(buf, sizeof buf, "\",\"ph\":\"X\",\"pid\":%d,\"tid\":%d,\"ts\":%.3f,\"dur\":%.3f},\n", R.rank,
                          track, t0 * 1e6, (t1 - t0) * 1e6);
            mine += buf;
        };
        for (auto& h : trace_rt::g_host) ev(h.name, 4, h.t0, h.t1);
        for (auto& d : trace_rt::g_resolved) ev(d.name, d.track, d.t0, d.t1);
        for (int t = 0; t < 5; ++t) {
            std::snprintf(buf, sizeof buf,
                          "{\"name\":\"thread_name\",\"ph\":\"M\",\"pid\":%d,\"tid\":%d,\"args\":{\"name\":\"%s\"}},\n",
                          R.rank, t, trace_rt::track_name(t));
            mine += buf;
        }
        std::snprintf(buf, sizeof buf,
                      "{\"name\":\"process_name\",\"ph\":\"M\",\"pid\":%d,\"args\":{\"name\":\"rank %d\"}},\n", R.rank,
                      R.rank);
        mine += buf;
        trace_rt::g_host.clear();
        trace_rt::g_resolved.clear();
    }
    // gather to rank 0: lengths, then every rank's text padded to the longest
    std::string all = mine;
    if (R.size > 1) {
        Comm* w = world_comm();
        hipStream_t s = R.main;
        Scratch len(sizeof(int64_t), s), lens(sizeof(int64_t) * R.size, s);
        const int64_t n = (int64_t)mine.size();
        upload(len.p, &n, sizeof n, s);
        w->allgather(len.p, lens.p, sizeof(int64_t), s);
        std::vector<int64_t> hl((size_t)R.size);
        NHIP(hipMemcpyAsync(hl.data(), lens.p, sizeof(int64_t) * R.size, hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
        int64_t mx = 1;
        for (auto v : hl) mx = std::max(mx, v);
        std::vector<char> pad((size_t)mx, ' ');
        std::copy(mine.begin(), mine.end(), pad.begin());
        Scratch sb((size_t)mx, s), rb((size_t)mx * R.size, s);
        upload(sb.p, pad.data(), (size_t)mx, s);
        w->allgather(sb.p, rb.p, (size_t)mx, s);
        std::vector<char> h((size_t)mx * R.size);
        NHIP(hipMemcpyAsync(h.data(), rb.p, h.size(), hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
        all.clear();
        for (int r = 0; r < R.size; ++r) all.append(h.data() + (size_t)r * mx, (size_t)hl[r]);
    }
    if (R.rank != 0) return;
    // drop the trailing ",\n"
    while (!all.empty() && (all.back() == '\n' || all.back() == ',' || all.back() == ' ')) all.pop_back();
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) throw Error("trace::finish: cannot write " + path);
    std::fprintf(f, "{\"traceEvents\":[\n%s\n],\"displayTimeUnit\":\"ms\",\"otherData\":{\"library\":\"%s\"}}\n",
                 all.c_str(), version());
    std::fclose(f);
}

}  // namespace trace

std::map<std::string, double> timers() {
    std::lock_guard<std::mutex> lk(trace_rt::g_mu);
    if (!trace_rt::g_dev.empty()) trace_rt::resolve_locked();
    return trace_rt::g_timers;
}

void clear_timers() {
    std::lock_guard<std::mutex> lk(trace_rt::g_mu);
    trace_rt::g_timers.clear();
}

}  // namespace native
}  // namespace slate_amd
