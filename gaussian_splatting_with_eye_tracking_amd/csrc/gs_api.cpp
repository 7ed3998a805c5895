// gs_api.cpp -- C-ABI entry points (include/gsplat_amd.h): stage
// orchestration on one HIP stream.
//
// Base forward follows base/cr/rasterizer_impl.cu:198-336, backward :340-434,
// markVisible :141-153; the AMR forward amr/cr/rasterizer_impl.cu:296-694;
// simple-knn knn/simple_knn.cu:185-221.  Differences that are deliberate
// (all documented in DESIGN.md):
//   * everything runs on the caller's stream (the reference uses the legacy
//     default stream);
//   * one blocking 16-byte read-back per forward (K plus the error and
//     large-tile words) -- the reference does 1 (base) / 4 (AMR step 0) plus a
//     cudaMalloc/cudaFree pair;
//   * simple-knn has no host synchronisation at all (the reference has 2).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <functional>
#include <algorithm>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

#include "../../include/gsplat_amd.h"
#include "gs_kernels.h"
#include "gs_layout.h"

using namespace gsamd;

namespace {

thread_local std::string g_err;


struct GsError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define GS_HIP_NOTHROW(expr) (void)(expr)
#define GS_HIP(expr)                                                                                  \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            throw GsError(std::string(#expr) + " failed: " + hipGetErrorString(_e) + " at " __FILE__ \
                          ":" + std::to_string(__LINE__));                                            \
    } while (0)

// ---- optional per-stage timing (gs_profile_*): hipEvents recorded on the
// launch stream around each stage; elapsed times are harvested lazily.
constexpr int kStages = 15;
const char* kStageNames[kStages] = {"preprocess", "tile_scan",    "duplicate",   "sort_tiles",
                                    "render",     "render_bwd",   "bwd_gauss",   "amr_levels",
                                    "amr_render", "amr_interp",   "knn",         "zero_accum",
                                    "count_tiles", "multiview_bwd", "amr_lists"};
enum Stage {
    kPre, kScan, kDup, kSort, kRender, kRenderBwd, kBwdGauss, kAmrLevels, kAmrRender, kAmrInterp, kKnn, kZero, kCount,
    kMultiView, kAmrLists
};
struct Profiler {
    bool on = false;
    uint32_t mask = ~0u;  // stages that record events (bit = Stage)
    struct Pending { int stage; hipEvent_t a, b; };
    std::vector<Pending> pending;
    double total_ms[kStages] = {0};
    long count[kStages] = {0};
    std::vector<hipEvent_t> pool;
    hipEvent_t get() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e; GS_HIP_NOTHROW(hipEventCreate(&e)); return e;
    }
    void harvest() {
        for (auto& p : pending) {
            float ms = 0.f;
            if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
                total_ms[p.stage] += ms; count[p.stage] += 1;
            }
            pool.push_back(p.a); pool.push_back(p.b);
        }
        pending.clear();
    }
};
Profiler g_prof;
std::mutex g_prof_mu;

// on_dispatch (single-kernel stages whose launcher takes the pair with
// take_dispatch_events): the events are recorded by the kernel's own dispatch
// (hipExtLaunchKernelGGL start / stop events) instead of two marker packets
// around it -- the markers cost ~6 us of idle queue each around a timed
// kernel (profiles/r05a_gaptrace: 5.9 + 6.1 us per step around render_bwd).
thread_local DispatchEvents t_dispatch;

struct StageTimer {
    int stage; hipStream_t s; hipEvent_t a = nullptr, b = nullptr; bool on_dispatch;
    StageTimer(int st, hipStream_t str, bool dispatch = false) : stage(st), s(str), on_dispatch(dispatch) {
        if (!g_prof.on || !((g_prof.mask >> st) & 1u)) return;
        std::lock_guard<std::mutex> l(g_prof_mu);
        a = g_prof.get(); b = g_prof.get();
        if (on_dispatch) t_dispatch = DispatchEvents{a, b};
        else hipEventRecord(a, s);
    }
    ~StageTimer() {
        if (!a) return;
        if (on_dispatch) {
            const bool taken = t_dispatch.start == nullptr;  // (the launcher cleared it)
            t_dispatch = DispatchEvents{};
            std::lock_guard<std::mutex> l(g_prof_mu);
            if (taken) {
                g_prof.pending.push_back({stage, a, b});
            } else {  // no kernel was launched: nothing to time
                g_prof.pool.push_back(a);
                g_prof.pool.push_back(b);
            }
            return;
        }
        hipEventRecord(b, s);
        std::lock_guard<std::mutex> l(g_prof_mu);
        g_prof.pending.push_back({stage, a, b});
    }
};

// CHECK_CUDA(A, debug) equivalent (base/cr/auxiliary.h:166-173): in debug
// mode synchronise after every stage and raise on the first error.
void stage_check(bool debug, hipStream_t s, const char* stage) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug) e = hipStreamSynchronize(s);
    if (e != hipSuccess) throw GsError(std::string("[HIP ERROR] in stage ") + stage + ": " + hipGetErrorString(e));
}

// Pinned 64-B landing zone for the single read-back per forward.
uint32_t* pinned_words() {
    thread_local uint32_t* p = nullptr;
    if (!p) {
        void* q = nullptr;
        GS_HIP(hipHostMalloc(&q, 64, hipHostMallocDefault));
        p = static_cast<uint32_t*>(q);
    }
    return p;
}

// Mapped, coherent host words the tile scan writes the header into (no copy
// kernel): thread-local like pinned_words; (host pointer, device pointer).
// 0: copy + event; 1: scan-stored words + event; 2 (default): scan-stored
// words + token, polled by the host (config 3 frame 0.575 -> 0.536 ms, config 2
// 0.971 -> 0.965 ms per step, profiles/r03m_ab_hdr_mirror.log)
// set_tuning("hdr_mirror"): 2 (default) the polled read-back -- the tile scan
// stores the header words and a per-call token into mapped host memory and
// the host spins on the token (no event or copy between the scan and the
// work behind it: config 3 frame 0.575 -> 0.536 ms, profiles/r03m_ab_hdr_mirror.log);
// 0 (fallback) a copy + event behind the scan.  (The mirror waited for by an
// event, and the copy on a side stream, measured no faster: r02q / r02p;
// removed.)  -1: GSAMD_HDR_MIRROR, else 2.
int g_hdr_mirror = -1;

bool hdr_mirror_on() {
    if (g_hdr_mirror < 0) {
        const char* e = std::getenv("GSAMD_HDR_MIRROR");
        g_hdr_mirror = (e && std::atoi(e) == 0) ? 0 : 2;
    }
    return g_hdr_mirror != 0;
}

std::pair<uint32_t*, uint32_t*> mirror_words() {
    thread_local uint32_t* h = nullptr;
    thread_local uint32_t* d = nullptr;
    if (!h) {
        void* q = nullptr;
        GS_HIP(hipHostMalloc(&q, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
        void* dq = nullptr;
        GS_HIP(hipHostGetDevicePointer(&dq, q, 0));
        h = static_cast<uint32_t*>(q);
        d = static_cast<uint32_t*>(dq);
    }
    return {h, d};
}

void read_header(const uint32_t* hdr_dev, uint32_t out[4], hipStream_t s) {
    uint32_t* h = pinned_words();
    GS_HIP(hipMemcpyAsync(h, hdr_dev, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    std::memcpy(out, h, 4 * sizeof(uint32_t));
}

// The same read-back in two halves: the copy (and an event behind it) is
// enqueued, the caller enqueues work that does not depend on K, then waits for
// the copy alone -- that work runs while the host reacts to K.  With the
// polled mirror (hdr_mirror 2) the scan stores the words into host memory
// itself, followed by a per-call token the host spins on.
thread_local uint32_t t_mirror_token = 0;
uint32_t next_mirror_token() {
    t_mirror_token = t_mirror_token + 1u ? t_mirror_token + 1u : 1u;
    return t_mirror_token;
}

hipEvent_t& copy_done_event() {
    thread_local std::vector<hipEvent_t> per_device;
    int dev = 0;
    GS_HIP(hipGetDevice(&dev));
    if ((int)per_device.size() <= dev) per_device.resize(dev + 1, nullptr);
    if (!per_device[dev]) GS_HIP(hipEventCreateWithFlags(&per_device[dev], hipEventDisableTiming));
    return per_device[dev];
}

void begin_header_read(const uint32_t* hdr_dev, hipStream_t s, const uint32_t* mirror = nullptr) {
    if (mirror) return;  // the scan stores the words into host memory itself
    GS_HIP(hipMemcpyAsync(pinned_words(), hdr_dev, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GS_HIP(hipEventRecord(copy_done_event(), s));
}

void finish_header_read(uint32_t out[4], const uint32_t* mirror = nullptr, hipStream_t s = nullptr,
                        const uint32_t* hdr_dev = nullptr) {
    if (mirror) {
        const volatile uint32_t* m = mirror;
        auto token = [&]() { return __atomic_load_n(const_cast<const uint32_t*>(mirror) + 4, __ATOMIC_ACQUIRE); };
        const auto t0 = std::chrono::steady_clock::now();
        uint64_t spins = 0;
        while (token() != t_mirror_token) {
            __builtin_ia32_pause();  // (a spin-wait hint: the wait is ~10-50 us)
            // a stream that faulted or was never run: wait for it, then re-check once
            if ((++spins & 0xffff) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                GS_HIP(hipStreamSynchronize(s));
                if (token() != t_mirror_token)
                    throw GsError("header read-back: the tile scan did not publish its token");
                break;
            }
        }
        for (int i = 0; i < 4; i++) out[i] = m[i];
        // seqlock check: the words and the token share this thread's slot, so a
        // scan of an earlier call that is still queued on another stream (its
        // caller never finished, e.g. an exception in between) could rewrite
        // them after the token test above.  Then the token is no longer ours:
        // fall back to the device's own header words, after this stream.
        if (token() != t_mirror_token) {
            if (!hdr_dev) throw GsError("header read-back: the mirror slot was overwritten");
            GS_HIP(hipStreamSynchronize(s));
            GS_HIP(hipMemcpy(out, hdr_dev, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost));
        }
        return;
    }
    GS_HIP(hipEventSynchronize(copy_done_event()));
    std::memcpy(out, pinned_words(), 4 * sizeof(uint32_t));
}

// Geometry buffers whose grad_accum rows the forward render zeroed and no
// backward has consumed yet (keyed by the rows' address): the first backward
// after such a forward skips its memset, any other zeroes the rows itself --
// a second backward of one forward (retain_graph), an AMR geometry buffer
// (the AMR forward does not zero them), a forward that could not fuse the zeroing.
std::mutex g_clean_mu;
std::unordered_set<const float*> g_accum_clean;

// Geometry buffers whose forward stored d(rgb)/d(dir) (keyed by the rows'
// address; set or cleared by every forward): the backward then launches the
// drgb-known bwd_gauss kernel (no SH-coefficient path compiled in).
// Bounded: the newest kDrgbEntries forwards' buffers (an entry older than that
// only costs the drgb-known kernel; its device-side header check keeps a
// stale entry correct either way).
constexpr size_t kDrgbEntries = 64;
std::mutex g_drgb_mu;
std::deque<const float*> g_drgb_rows;
void set_drgb_written(const float* rows, bool w) {
    std::lock_guard<std::mutex> l(g_drgb_mu);
    g_drgb_rows.erase(std::remove(g_drgb_rows.begin(), g_drgb_rows.end(), rows), g_drgb_rows.end());
    if (!w) return;
    g_drgb_rows.push_back(rows);
    if (g_drgb_rows.size() > kDrgbEntries) g_drgb_rows.pop_front();
}
bool drgb_written(const float* rows) {
    std::lock_guard<std::mutex> l(g_drgb_mu);
    return std::find(g_drgb_rows.begin(), g_drgb_rows.end(), rows) != g_drgb_rows.end();
}

void set_accum_clean(const float* rows, bool clean) {
    std::lock_guard<std::mutex> l(g_clean_mu);
    if (clean) g_accum_clean.insert(rows);
    else g_accum_clean.erase(rows);
}

bool take_accum_clean(const float* rows) {
    std::lock_guard<std::mutex> l(g_clean_mu);
    return g_accum_clean.erase(rows) > 0;
}

void zero_accum_unless_clean(const GeomView& g, int P, hipStream_t s) {
    if (take_accum_clean(g.grad_accum)) return;
    StageTimer _t(kZero, s);
    GS_HIP(hipMemsetAsync(g.grad_accum, 0, sizeof(float) * kGradRow * (size_t)P, s));
}

// Per-call options of this thread's forwards (gs_set_thread_option; thread-
// local, so concurrent callers on other threads are unaffected):
//   fwd_zero (1): the forward render zeroes the backward's accumulator rows
//     behind the blend when a backward can follow; 0: the backward memsets them;
//   sh_drgb (1): the preprocess stores d(rgb)/d(dir) of the SH colours
//     (GeomView::drgb, 36 B per visible Gaussian) and the backward reads them
//     instead of the 192-B SH rows; 0: the backward reads the coefficients;
//   store_cov3d (0): the preprocess writes the geometry buffer's cov3D (the
//     parity tests read it; nothing in the path does);
//   fwd_no_grad: one-shot -- the NEXT forward on this thread needs no
//     backward (below).
thread_local int t_fwd_zero = 1;
thread_local int t_sh_drgb = 1;
thread_local int t_store_cov3d = 0;
// Capacity for the speculative duplicate: the last base forward's K plus
// 1/8 (0 before the first call, or when speculation is switched off).
int g_spec_dup = 1;  // set_tuning("spec_dup")
// The speculative duplicate's capacity, remembered per (device, W, H, P):
// workloads that alternate render sizes or scenes (train 1080p / eval
// thumbnails) keep one prediction each instead of over-sizing the small
// renders and missing on the large ones.  A few entries per thread, least
// recently used replaced; an unknown key runs the synchronous path.
struct SpecKey {
    int dev, W, H, P;
    bool operator==(const SpecKey& o) const { return dev == o.dev && W == o.W && H == o.H && P == o.P; }
};
struct SpecEntry {
    SpecKey key;
    size_t cap;
    uint64_t used;
};
constexpr int kSpecEntries = 8;
thread_local SpecEntry t_spec[kSpecEntries] = {};
thread_local uint64_t t_spec_clock = 0;
SpecKey spec_key(int W, int H, int P) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    return SpecKey{dev, W, H, P};
}
size_t spec_capacity(const SpecKey& k) {
    if (!g_spec_dup) return 0;
    for (SpecEntry& e : t_spec)
        if (e.cap && e.key == k) {
            e.used = ++t_spec_clock;
            return e.cap;
        }
    return 0;
}
void note_k(const SpecKey& k, int K) {
    const size_t cap = K > 0 ? (size_t)K + (size_t)K / 8 + 4096 : 0;
    SpecEntry* victim = &t_spec[0];
    for (SpecEntry& e : t_spec) {
        if (e.cap && e.key == k) { victim = &e; break; }
        if (!e.cap || e.used < victim->used) victim = &e;
    }
    victim->key = k;
    victim->cap = cap;
    victim->used = ++t_spec_clock;
}

char* call_resize(const gs_buffer& b, size_t n, const char* what) {
    if (!b.resize) throw GsError(std::string("no resize callback for ") + what);
    char* p = b.resize(b.ctx, n);
    if (!p && n > 0) throw GsError(std::string("resize failed for ") + what);
    if (reinterpret_cast<uintptr_t>(p) % 16 != 0) throw GsError(std::string("unaligned buffer for ") + what);
    return p;
}

template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    } catch (...) {
        g_err = "unknown error";
        return -1;
    }
}

struct ForwardIn {
    int P, D, M;
    const float *background, *means3D, *shs, *colors_precomp, *opacities, *scales, *rotations, *cov3D_precomp,
        *viewmatrix, *projmatrix, *cam_pos;
    int width, height;
    float scale_modifier, tan_fovx, tan_fovy;
    int prefiltered;
};

// Per-call token for the header's error word (never 0: a zeroed header at
// T == 0 must not read as an error).
// Drawn from one process-wide counter (hashed), so no two calls -- on any
// thread -- share a token, and a stale word left by another call never reads
// as this call's error.
uint32_t next_error_token() {
    static std::atomic<uint32_t> counter{0};
    uint32_t t = counter.fetch_add(1u, std::memory_order_relaxed) + 1u;
    t ^= t >> 16; t *= 0x7feb352du; t ^= t >> 15; t *= 0x846ca68bu; t ^= t >> 16;  // bijective mix
    return t ? t : 1u;
}

// gs_set_thread_option("fwd_no_grad", 1): the NEXT forward on this thread is
// known to need no backward (the autograd wrappers under no_grad / with no
// input requiring a gradient): its preprocess skips the SH-derivative rows
// only the backward reads (the header flag kHdrDrgb then says so, and a
// backward would fall back to the SH coefficients).  One-shot: every forward
// entry consumes it.
thread_local int t_fwd_no_grad = 0;
bool take_fwd_no_grad() {
    const bool v = t_fwd_no_grad != 0;
    t_fwd_no_grad = 0;
    return v;
}
thread_local bool t_store_drgb = true;  // this forward's choice (take_fwd_no_grad)
// gs_set_thread_option("amr_step0_unfilled", 1): one-shot -- the NEXT AMR
// forward on this thread, if at foveaStep 0, leaves its image unwritten: the
// caller overwrites every pixel (gs_amr_accumulate_step with
// GSPLAT_AMD_AMR_STEPS_1_TO_4_FILL), so step 0's 3 x H x W zero fill is skipped.
// Every AMR forward entry consumes it.
thread_local int t_amr_step0_unfilled = 0;

PreprocessArgs make_pp(const ForwardIn& in, int tile) {
    PreprocessArgs a;
    a.P = in.P;
    a.D = in.D;
    a.M = in.M;
    a.means3D = in.means3D;
    a.scales = in.scales;
    a.scale_modifier = in.scale_modifier;
    a.rotations = in.rotations;
    a.opacities = in.opacities;
    a.shs = in.shs;
    a.cov3D_precomp = in.cov3D_precomp;
    a.colors_precomp = in.colors_precomp;
    a.viewmatrix = in.viewmatrix;
    a.projmatrix = in.projmatrix;
    a.cam_pos = in.cam_pos;
    a.W = in.width;
    a.H = in.height;
    a.tan_fovx = in.tan_fovx;
    a.tan_fovy = in.tan_fovy;
    // rasterizer_impl.cu:222-223 (float arithmetic)
    a.focal_y = (float)in.height / (2.0f * in.tan_fovy);
    a.focal_x = (float)in.width / (2.0f * in.tan_fovx);
    a.block = tile;
    a.prefiltered = in.prefiltered;
    a.store_cov3d = t_store_cov3d;
    a.store_drgb = t_sh_drgb && t_store_drgb;
    a.zero_words = nullptr;
    a.zero_n = 0;
    a.err_token = 0;
    return a;
}

struct Binned {
    GeomView g;
    ImageView img;
    BinningView b;
    AmrBinningView ab;  // tile == 32 only
    int K;
    int T;
    int* radii;
};

// preprocess -> tile scan -> (K read-back) -> duplicate -> per-tile sort.
// `before_k`: work that needs the scan but not K, enqueued behind the K copy
// and run while the host waits for it.
Binned preprocess_and_bin(const ForwardIn& in, const gs_buffer& geometry, const gs_buffer& binning,
                          const gs_buffer& image, int* radii, int tile, bool debug, hipStream_t s,
                          const std::function<void(Binned&)>& before_k = nullptr, int fused_sort_max = 0) {
    Binned r;
    const int W = in.width, H = in.height;
    const int gx = (W + tile - 1) / tile, gy = (H + tile - 1) / tile;
    r.T = gx * gy;
    const size_t N = (size_t)W * H;
    // the optional tail (gs_layout.h) only when this forward writes into it
    const bool tail = t_store_cov3d || (in.colors_precomp == nullptr && t_sh_drgb && t_store_drgb);
    char* gbase = call_resize(geometry, carve_geom(nullptr, in.P, nullptr, tail, tile == 32), "geometry");
    carve_geom(gbase, in.P, &r.g);
    set_accum_clean(r.g.grad_accum, false);  // this forward decides afresh
    char* ibase = call_resize(image, carve_image(nullptr, N, r.T, nullptr, tile), "image");
    carve_image(ibase, N, r.T, &r.img, tile);
    r.radii = radii ? radii : r.g.radii;
    // The header needs no zeroing: the tile scan stores K and the tile
    // statistics, and a prefiltered violation stores this call's token in the
    // error word (stale words never equal it).  With the LDS-privatised count
    // the preprocess zeroes the tile histogram; otherwise it adds into it.
    const bool lds_bin = r.T <= kLdsTiles;
    if (r.T == 0) GS_HIP(hipMemsetAsync(r.g.hdr, 0, kHdrWords * sizeof(uint32_t), s));
    if (r.T > 0 && !lds_bin) GS_HIP(hipMemsetAsync(r.img.tile_count, 0, sizeof(uint32_t) * kBinSlots * r.T, s));
    PreprocessArgs pa = make_pp(in, tile);
    pa.err_token = next_error_token();
    set_drgb_written(r.g.drgb, pa.store_drgb && in.colors_precomp == nullptr);
    if (r.T > 0 && lds_bin) {
        pa.zero_words = r.img.tile_count;
        pa.zero_n = kBinSlots * r.T;
    }
    { StageTimer _t(kPre, s); launch_preprocess(pa, r.g, r.radii, lds_bin ? nullptr : r.img.tile_count, s); }
    stage_check(debug, s, "preprocess");
    if (lds_bin) { StageTimer _t(kCount, s); launch_count_tiles(in.P, r.g, r.radii, W, H, tile, r.img, s); }
    stage_check(debug, s, "count_tiles");
    const std::pair<uint32_t*, uint32_t*> mirror =
        (r.T > 0 && hdr_mirror_on()) ? mirror_words() : std::pair<uint32_t*, uint32_t*>{nullptr, nullptr};
    const bool amr = tile == 32;  // the AMR layout appends records and region lists
    // Base forward: the duplicate is launched speculatively into a binning
    // buffer sized for the capacity the last calls suggest, before K is on
    // the host, so the GPU runs it while the host waits for K instead of
    // idling through the read-back (~25 us per view at config 2).  The
    // kernel does nothing if K > capacity; then the buffer is re-sized for K
    // and the duplicate relaunched.  Only point_list (offset 0) outlives the
    // forward, so a buffer carved for capacity >= K serves the backward as is.
    bool dup_done = false;
    const SpecKey skey = spec_key(W, H, in.P);
    const size_t cap = (!amr && !before_k && r.T > 0 && !debug) ? spec_capacity(skey) : 0;
    // the polled read-back's words: published by the speculative duplicate's
    // first thread when there is one (binning.hip publish_header), else by the
    // scan
    const uint32_t mtoken = mirror.second ? next_mirror_token() : 0u;
    const bool pub_dup = cap > 0 && mirror.second != nullptr;
    if (r.T > 0) { StageTimer _t(kScan, s); launch_tile_scan(r.T, r.img, r.g.hdr, s, pub_dup ? nullptr : mirror.second, bin_slots_for(in.P, gx, gy, tile), gx, dup_banded(gx, gy, tile), pub_dup ? 0u : mtoken); }
    stage_check(debug, s, "tile_scan");
    uint32_t hdr[4];
    if (before_k) {
        begin_header_read(r.g.hdr, s, mirror.first);
        before_k(r);
        finish_header_read(hdr, mirror.first, s, r.g.hdr);
    } else if (cap > 0) {
        begin_header_read(r.g.hdr, s, mirror.first);
        char* sbase = call_resize(binning, carve_binning(nullptr, cap, nullptr), "binning");
        carve_binning(sbase, cap, &r.b);
        { StageTimer _t(kDup, s); launch_duplicate(in.P, r.g, r.radii, W, H, tile, r.img, r.b, s, (uint32_t)cap, r.g.hdr, (uint32_t)cap, pub_dup ? mirror.second : nullptr, pub_dup ? mtoken : 0u); }
        finish_header_read(hdr, mirror.first, s, r.g.hdr);
        dup_done = hdr[kHdrNumRendered] <= cap;
    } else if (mirror.first) {
        begin_header_read(r.g.hdr, s, mirror.first);
        finish_header_read(hdr, mirror.first, s, r.g.hdr);
    } else {
        read_header(r.g.hdr, hdr, s);
    }
    if (in.prefiltered && hdr[kHdrError] == pa.err_token)
        throw GsError("Point is filtered although prefiltered is set. This shouldn't happen!");
    r.K = (int)hdr[kHdrNumRendered];
    if (!amr) note_k(skey, r.K);
    if (!dup_done) {
        char* bbase = call_resize(binning, carve_binning(nullptr, r.K, nullptr, nullptr, amr), "binning");
        carve_binning(bbase, r.K, &r.b, amr ? &r.ab : nullptr);
    }
    if (r.K > 0) {
        if (!dup_done) { StageTimer _t(kDup, s); launch_duplicate(in.P, r.g, r.radii, W, H, tile, r.img, r.b, s, (uint32_t)r.K); }
        stage_check(debug, s, "duplicate");
        { StageTimer _t(kSort, s); launch_sort_tiles(r.T, r.img, r.b, (int)hdr[kHdrMaxTileCount], (int)hdr[kHdrNumLargeTiles], s, fused_sort_max); }
        stage_check(debug, s, "sort_tiles");
    }
    return r;
}

}  // namespace

DispatchEvents gsamd::take_dispatch_events() {
    const DispatchEvents e = t_dispatch;
    t_dispatch = DispatchEvents{};
    return e;
}

extern "C" {

int gs_abi_version(void) { return GSPLAT_AMD_ABI_VERSION; }

// build.py passes -DGSAMD_DIGEST="<source_digest()>" for this file
#ifndef GSAMD_DIGEST
#define GSAMD_DIGEST "unstamped"
#endif
const char* gs_build_digest(void) { return GSAMD_DIGEST; }

const char* gs_last_error(void) { return g_err.c_str(); }

int gs_rasterizer_forward(gs_buffer geometry, gs_buffer binning, gs_buffer image, int P, int D, int M,
                          const float* background, int width, int height, const float* means3D, const float* shs,
                          const float* colors_precomp, const float* opacities, const float* scales,
                          float scale_modifier, const float* rotations, const float* cov3D_precomp,
                          const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                          float tan_fovy, int prefiltered, float* out_color, int* radii, int debug, void* stream) {
    t_store_drgb = !take_fwd_no_grad();
    return guarded([&]() -> int {
        if (P <= 0) return 0;
        hipStream_t s = static_cast<hipStream_t>(stream);
        ForwardIn in{P, D, M, background, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                     viewmatrix, projmatrix, cam_pos, width, height, scale_modifier, tan_fovx, tan_fovy, prefiltered};
        Binned r = preprocess_and_bin(in, geometry, binning, image, radii, 16, debug != 0, s);
        const float* feats = colors_precomp ? colors_precomp : r.g.rgb;
        bool zeroed;
        {
            StageTimer _t(kRender, s, true);
            // the accumulator rows are zeroed behind the blend only when a
            // backward can follow (not under the forward-only hint: a later
            // backward of this forward then zeroes them itself)
            const bool zero = t_fwd_zero && t_store_drgb;
            zeroed = launch_render_forward(width, height, r.img, r.b, r.g, feats, background, out_color, s,
                                           zero ? r.g.grad_accum : nullptr, zero ? (size_t)kGradRow * (size_t)P : 0,
                                           reinterpret_cast<uint8_t*>(r.b.scratch));
        }
        if (zeroed) set_accum_clean(r.g.grad_accum, true);
        stage_check(debug != 0, s, "render");
        return r.K;
    });
}

namespace {
// Shared by the base and the AMR backward.  amr_mode 0: base 16-px tiles;
// != 0: AMR 32-px tiles, the rendered sub-lattices of foveaStep amr_mode
// (> 0) or of render_once (< 0; dL_dpix already folded through the
// interpolation when it was applied).
int rasterizer_backward_impl(int amr_mode, int P, int D, int M, int R, const float* background, int width,
                             int height, const float* means3D, const float* shs, const float* colors_precomp,
                             const float* scales, float scale_modifier, const float* rotations,
                             const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                             const float* campos, float tan_fovx, float tan_fovy, const int* radii, char* geom_buffer,
                             char* binning_buffer, char* img_buffer, const float* dL_dpix, float* dL_dmean2D,
                             float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D,
                             float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot, int debug,
                             hipStream_t s) {
    {
        if (P <= 0) return 0;
        const int tile = amr_mode != 0 ? 32 : 16;
        const int T = ((width + tile - 1) / tile) * ((height + tile - 1) / tile);
        GeomView g;
        ImageView img;
        BinningView b;
        carve_geom(geom_buffer, P, &g);
        carve_image(img_buffer, (size_t)width * height, T, &img, tile);
        carve_binning(binning_buffer, R, &b);
        if (!radii) radii = g.radii;
        zero_accum_unless_clean(g, P, s);
        const float* colors = colors_precomp ? colors_precomp : g.rgb;
        if (R > 0) {
            StageTimer _t(kRenderBwd, s, amr_mode == 0);
            if (amr_mode != 0) launch_amr_render_backward(width, height, amr_mode, img, b, g, colors, background, dL_dpix, s);
            else launch_render_backward(width, height, img, b, g, colors, background, dL_dpix, s, R);
        }
        stage_check(debug != 0, s, "render_backward");
        BackwardGaussArgs a;
        a.P = P;
        a.D = D;
        a.M = M;
        a.means3D = means3D;
        a.radii = radii;
        a.shs = shs;
        a.scales = scales;
        a.rotations = rotations;
        a.scale_modifier = scale_modifier;
        a.cov3D = cov3D_precomp ? cov3D_precomp : g.cov3D;
        a.viewmatrix = viewmatrix;
        a.projmatrix = projmatrix;
        a.campos = campos;
        a.focal_y = (float)height / (2.0f * tan_fovy);
        a.focal_x = (float)width / (2.0f * tan_fovx);
        a.tan_fovx = tan_fovx;
        a.tan_fovy = tan_fovy;
        a.has_cov_precomp = cov3D_precomp != nullptr;
        a.drgb = g.drgb;  // read only where the header says this forward wrote the rows
        a.drgb_known = a.drgb != nullptr && drgb_written(g.drgb);
        a.hdr = g.hdr;
        a.dL_dmean2D = dL_dmean2D;
        a.dL_dconic = dL_dconic;
        a.dL_dopacity = dL_dopacity;
        a.dL_dcolor = dL_dcolor;
        a.dL_dmean3D = dL_dmean3D;
        a.dL_dcov3D = dL_dcov3D;
        a.dL_dsh = dL_dsh;
        a.dL_dscale = dL_dscale;
        a.dL_drot = dL_drot;
        { StageTimer _t(kBwdGauss, s); launch_backward_gaussians(a, g, s); }
        stage_check(debug != 0, s, "preprocess_backward");
        return 0;
    }
}
}  // namespace

int gs_rasterizer_backward(int P, int D, int M, int R, const float* background, int width, int height,
                           const float* means3D, const float* shs, const float* colors_precomp, const float* scales,
                           float scale_modifier, const float* rotations, const float* cov3D_precomp,
                           const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                           float tan_fovy, const int* radii, char* geom_buffer, char* binning_buffer,
                           char* img_buffer, const float* dL_dpix, float* dL_dmean2D, float* dL_dconic,
                           float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
                           float* dL_dsh, float* dL_dscale, float* dL_drot, int debug, void* stream) {
    return guarded([&]() -> int {
        return rasterizer_backward_impl(0, P, D, M, R, background, width, height, means3D, shs, colors_precomp,
                                        scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix,
                                        campos, tan_fovx, tan_fovy, radii, geom_buffer, binning_buffer, img_buffer,
                                        dL_dpix, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, dL_dmean3D, dL_dcov3D,
                                        dL_dsh, dL_dscale, dL_drot, debug, static_cast<hipStream_t>(stream));
    });
}

int gs_amr_rasterizer_backward(int P, int D, int M, int R, const float* background, int width, int height,
                               const float* means3D, const float* shs, const float* colors_precomp,
                               const float* scales, float scale_modifier, const float* rotations,
                               const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                               const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                               char* geom_buffer, char* binning_buffer, char* img_buffer, int foveaStep,
                               int interpolate_image, const float* dL_dpix, float* dL_dpix_scratch,
                               float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor,
                               float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot,
                               int debug, void* stream) {
    return guarded([&]() -> int {
        if (foveaStep == 0) throw GsError("gs_amr_rasterizer_backward: foveaStep 0 renders nothing");
        if (foveaStep > 4) throw GsError("gs_amr_rasterizer_backward: foveaStep 1..4 or < 0 (render_once)");
        if (interpolate_image && foveaStep > 0)
            throw GsError("gs_amr_rasterizer_backward: interpolate_image is supported for render_once only");
        hipStream_t s = static_cast<hipStream_t>(stream);
        const float* g = dL_dpix;
        if (interpolate_image && P > 0) {
            if (!dL_dpix_scratch) throw GsError("gs_amr_rasterizer_backward: interpolation needs dL_dpix_scratch");
            const int T = ((width + 31) / 32) * ((height + 31) / 32);
            ImageView img;
            carve_image(img_buffer, (size_t)width * height, T, &img, 32);
            launch_amr_interp_fold(width, height, img, dL_dpix, dL_dpix_scratch, s);
            stage_check(debug != 0, s, "amr_interp_fold");
            g = dL_dpix_scratch;
        }
        return rasterizer_backward_impl(foveaStep, P, D, M, R, background, width, height, means3D, shs,
                                        colors_precomp, scales, scale_modifier, rotations, cov3D_precomp, viewmatrix,
                                        projmatrix, campos, tan_fovx, tan_fovy, radii, geom_buffer, binning_buffer,
                                        img_buffer, g, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, dL_dmean3D,
                                        dL_dcov3D, dL_dsh, dL_dscale, dL_drot, debug, s);
    });
}

int gs_rasterizer_backward_view_grads(int P, int R, const float* background, int width, int height,
                                      const float* colors_precomp, const float* viewmatrix, const float* projmatrix,
                                      const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                                      char* geom_buffer, char* binning_buffer, char* img_buffer,
                                      const float* dL_dpix, float* out_record, int debug, void* stream) {
    return guarded([&]() -> int {
        if (P < 0) throw GsError("gs_rasterizer_backward_view_grads: negative P");
        hipStream_t s = static_cast<hipStream_t>(stream);
        const int tile = 16;
        const int T = ((width + tile - 1) / tile) * ((height + tile - 1) / tile);
        GeomView g;
        ImageView img;
        BinningView b;
        carve_geom(geom_buffer, P, &g);
        carve_image(img_buffer, (size_t)width * height, T, &img, tile);
        carve_binning(binning_buffer, R, &b);
        if (!radii) radii = g.radii;
        zero_accum_unless_clean(g, P, s);
        const float* colors = colors_precomp ? colors_precomp : g.rgb;
        if (R > 0 && P > 0) { StageTimer _t(kRenderBwd, s, true); launch_render_backward(width, height, img, b, g, colors, background, dL_dpix, s, R); }
        stage_check(debug != 0, s, "render_backward");
        launch_pack_view_grads(P, g, radii, colors_precomp == nullptr, viewmatrix, projmatrix, campos, width, height,
                               tan_fovx, tan_fovy, out_record, s);
        stage_check(debug != 0, s, "pack_view_grads");
        return 0;
    });
}

namespace {
// The view table of a call with more than kMaxViews views: pinned host staging
// and a device copy, one pair per (thread, device), reused by every such call
// -- no allocation, no stream synchronisation per call.  `done` (recorded
// behind the kernel that reads the table) guards the reuse: the next call's
// host writes wait for it, and its stream waits for it before the copy
// overwrites the device table another stream's kernel may still read.
struct ViewTable {
    const float** host = nullptr;
    const float** dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
};

ViewTable& view_table(size_t n, hipStream_t s) {
    thread_local std::vector<ViewTable> per_device;
    int d = 0;
    GS_HIP(hipGetDevice(&d));
    if ((int)per_device.size() <= d) per_device.resize(d + 1);
    ViewTable& t = per_device[d];
    if (!t.done) GS_HIP(hipEventCreateWithFlags(&t.done, hipEventDisableTiming));
    GS_HIP(hipEventSynchronize(t.done));  // the last use's copy and kernel are done (a fresh event: at once)
    if (t.cap < n) {
        if (t.host) GS_HIP(hipHostFree(t.host));
        if (t.dev) GS_HIP(hipFree(t.dev));
        t.host = nullptr;
        t.dev = nullptr;
        t.cap = 0;
        void* h = nullptr;
        void* dv = nullptr;
        GS_HIP(hipHostMalloc(&h, n * sizeof(const float*), hipHostMallocDefault));
        t.host = static_cast<const float**>(h);
        GS_HIP(hipMalloc(&dv, n * sizeof(const float*)));
        t.dev = static_cast<const float**>(dv);
        t.cap = n;
    }
    GS_HIP(hipStreamWaitEvent(s, t.done, 0));
    return t;
}

// rows[v] / cams[v]: view v's row of Gaussian g0 and its camera, summed in v order
int multiview_impl(int P, int g0, int count, int D, int M, int V, const float* const* rows, const float* const* cams,
                   const float* means3D, const float* shs, const float* scales, const float* rotations,
                   float scale_modifier, float* dL_dmeans3D, float* dL_dsh, float* dL_dopacity, float* dL_dscales,
                   float* dL_drotations, float* grad_norm_accum, float* denom, float* max_radii, void* stream) {
    return guarded([&]() -> int {
        if (P <= 0 || count == 0) return 0;
        if (V <= 0) throw GsError("gs_backward_gaussians_multiview: V must be >= 1");
        if (g0 < 0 || count < 0 || g0 + count > P) throw GsError("gs_backward_gaussians_multiview: bad range");
        if (!scales || !rotations)
            throw GsError("gs_backward_gaussians_multiview: scales and rotations are required (no cov3D_precomp)");
        if (shs && (M <= 0 || M > 16 || D < 0 || D > 3))
            throw GsError("gs_backward_gaussians_multiview: SH with 1..16 coefficients, degree <= 3");
        if (grad_norm_accum && (!denom || !max_radii))
            throw GsError("gs_backward_gaussians_multiview: statistics need grad_norm_accum, denom and max_radii");
        MultiViewArgs a{};
        a.P = P; a.D = D; a.M = M; a.V = V;
        a.g0 = g0;
        a.count = count;
        for (int v = 0; v < V; v++)
            if (!rows[v] || !cams[v]) throw GsError("gs_backward_gaussians_multiview: null view row / camera");
        hipStream_t s = static_cast<hipStream_t>(stream);
        // up to kMaxViews views travel in the kernel arguments; more in a device
        // table (same kernel, same view order: bit-identical sums)
        ViewTable* vt = nullptr;
        if (V <= kMaxViews) {
            for (int v = 0; v < V; v++) {
                a.rows[v] = rows[v];
                a.cams[v] = cams[v];
            }
        } else {
            vt = &view_table(2 * (size_t)V, s);
            for (int v = 0; v < V; v++) {
                vt->host[v] = rows[v];
                vt->host[(size_t)V + v] = cams[v];
            }
            GS_HIP(hipMemcpyAsync(vt->dev, vt->host, 2 * (size_t)V * sizeof(const float*), hipMemcpyHostToDevice, s));
            // recorded at once, so a launch that throws below still leaves the
            // next call waiting for this copy before it rewrites (or frees) the
            // pinned staging the copy reads; recorded again after the kernel
            GS_HIP(hipEventRecord(vt->done, s));
            a.table = vt->dev;
        }
        a.means3D = means3D;
        a.shs = shs;
        a.scales = scales;
        a.rotations = rotations;
        a.scale_modifier = scale_modifier;
        a.dL_dmean3D = dL_dmeans3D;
        a.dL_dsh = dL_dsh;
        a.dL_dopacity = dL_dopacity;
        a.dL_dscale = dL_dscales;
        a.dL_drot = dL_drotations;
        a.grad_norm_accum = grad_norm_accum;
        a.denom = denom;
        a.max_radii = max_radii;
        { StageTimer _t(kMultiView, s); launch_multiview_backward(a, s); }
        if (vt) GS_HIP(hipEventRecord(vt->done, s));  // the staging and the table are free again after this
        stage_check(false, s, "multiview_backward");
        return 0;
    });
}

// strided views: view v's rows at rows + v * row_view_stride
int multiview_strided(int P, int g0, int count, int D, int M, int V, const float* rows, size_t row_view_stride,
                      const float* cams, size_t cam_stride, const float* means3D, const float* shs,
                      const float* scales, const float* rotations, float scale_modifier, float* dL_dmeans3D,
                      float* dL_dsh, float* dL_dopacity, float* dL_dscales, float* dL_drotations,
                      float* grad_norm_accum, float* denom, float* max_radii, void* stream) {
    std::vector<const float*> rp(V > 0 ? V : 0), cp(V > 0 ? V : 0);
    for (int v = 0; v < V; v++) {
        rp[v] = rows + (size_t)v * row_view_stride;
        cp[v] = cams + (size_t)v * cam_stride;
    }
    return multiview_impl(P, g0, count, D, M, V, rp.data(), cp.data(), means3D, shs, scales, rotations, scale_modifier,
                          dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales, dL_drotations, grad_norm_accum, denom,
                          max_radii, stream);
}
}  // namespace

int gs_backward_gaussians_multiview(int P, int D, int M, int V, const float* views, const float* means3D,
                                    const float* shs, const float* scales, const float* rotations,
                                    float scale_modifier, float* dL_dmeans3D, float* dL_dsh, float* dL_dopacity,
                                    float* dL_dscales, float* dL_drotations, float* grad_norm_accum, float* denom,
                                    float* max_radii, void* stream) {
    const size_t rec = (size_t)P * kViewRow + kCamWords;
    return multiview_strided(P, 0, P, D, M, V, views, rec, views + (size_t)P * kViewRow, rec, means3D, shs, scales,
                             rotations, scale_modifier, dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales, dL_drotations,
                             grad_norm_accum, denom, max_radii, stream);
}

int gs_backward_gaussians_multiview_range(int P, int g0, int count, int D, int M, int V, const float* rows,
                                          size_t row_view_stride, const float* cams, size_t cam_stride,
                                          const float* means3D, const float* shs, const float* scales,
                                          const float* rotations, float scale_modifier, float* dL_dmeans3D,
                                          float* dL_dsh, float* dL_dopacity, float* dL_dscales,
                                          float* dL_drotations, float* grad_norm_accum, float* denom,
                                          float* max_radii, void* stream) {
    return multiview_strided(P, g0, count, D, M, V, rows, row_view_stride, cams, cam_stride, means3D, shs, scales,
                             rotations, scale_modifier, dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales, dL_drotations,
                             grad_norm_accum, denom, max_radii, stream);
}

int gs_backward_gaussians_multiview_views(int P, int g0, int count, int D, int M, int V, const float* const* rows,
                                          const float* const* cams, const float* means3D, const float* shs,
                                          const float* scales, const float* rotations, float scale_modifier,
                                          float* dL_dmeans3D, float* dL_dsh, float* dL_dopacity, float* dL_dscales,
                                          float* dL_drotations, float* grad_norm_accum, float* denom,
                                          float* max_radii, void* stream) {
    if (!rows || !cams) {
        g_err = "gs_backward_gaussians_multiview_views: rows / cams arrays are required";
        return -1;
    }
    return multiview_impl(P, g0, count, D, M, V, rows, cams, means3D, shs, scales, rotations, scale_modifier,
                          dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales, dL_drotations, grad_norm_accum, denom,
                          max_radii, stream);
}

int gs_ritnet_conv(int ksize, int nseg, const float* const* in, const int* in_channels, const int* in_upsample,
                   int height, int width, const float* weight, const float* bias, int leaky_relu, const float* bn_scale,
                   const float* bn_shift, float* out, void* stream) {
    return guarded([&]() -> int {
        if (ksize != 1 && ksize != 3) throw GsError("gs_ritnet_conv: kernel size must be 1 or 3");
        if (nseg < 1 || nseg > 3) throw GsError("gs_ritnet_conv: 1 to 3 input segments");
        if ((bn_scale == nullptr) != (bn_shift == nullptr)) throw GsError("gs_ritnet_conv: bn_scale and bn_shift");
        for (int i = 0; i < nseg; i++)
            if (in_channels[i] <= 0 || !in[i] || (in_upsample[i] && ((height | width) & 1)))
                throw GsError("gs_ritnet_conv: bad input segment");
        if (height <= 0 || width <= 0) return 0;
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_ritnet_conv(ksize, in, in_channels, in_upsample, nseg, height, width, weight, bias, leaky_relu,
                           bn_scale, bn_shift, out, s);
        stage_check(false, s, "ritnet_conv");
        return 0;
    });
}

int gs_avgpool2(const float* in, int channels, int height, int width, float* out, void* stream) {
    return guarded([&]() -> int {
        if ((height | width) & 1) throw GsError("gs_avgpool2: even height and width required");
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_avgpool2(in, channels, height, width, out, s);
        stage_check(false, s, "avgpool2");
        return 0;
    });
}

int gs_ritnet_head(const float* in, int height, int width, const float* weight, const float* bias, float* logits,
                   uint8_t* labels, void* stream) {
    return guarded([&]() -> int {
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_ritnet_head(in, height, width, weight, bias, logits, labels, s);
        stage_check(false, s, "ritnet_head");
        return 0;
    });
}

int gs_label_moments(const uint8_t* labels, int height, int width, int label, double* out3, void* stream) {
    return guarded([&]() -> int {
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_label_moments(labels, height, width, label, out3, s);
        stage_check(false, s, "label_moments");
        return 0;
    });
}

int gs_eye_preprocess(const uint8_t* gray, int height, int width, const uint8_t* gamma_lut, double clip_limit,
                      int tiles_x, int tiles_y, float* luts, float* out, void* stream) {
    return guarded([&]() -> int {
        if (tiles_x <= 0 || tiles_y <= 0 || height % tiles_y || width % tiles_x)
            throw GsError("gs_eye_preprocess: image size must be divisible by the tile grid");
        if (height <= 0 || width <= 0) return 0;
        // OpenCV CLAHE_Impl::apply: int(clip * tile area / 256), at least 1; 0 disables clipping
        const int area = (width / tiles_x) * (height / tiles_y);
        int limit = 0;
        if (clip_limit > 0.0) {
            limit = static_cast<int>(clip_limit * area / 256);
            if (limit < 1) limit = 1;
        }
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_eye_preprocess(gray, height, width, gamma_lut, tiles_x, tiles_y, limit, luts, out, s);
        stage_check(false, s, "eye_preprocess");
        return 0;
    });
}

int gs_rasterizer_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                               uint8_t* present, void* stream) {
    return guarded([&]() -> int {
        launch_mark_visible(P, means3D, viewmatrix, projmatrix, reinterpret_cast<bool*>(present),
                            static_cast<hipStream_t>(stream));
        stage_check(false, static_cast<hipStream_t>(stream), "mark_visible");
        return 0;
    });
}

int gs_amr_rasterizer_forward(gs_buffer geometry, gs_buffer binning, gs_buffer image, int P, int D, int M,
                              const float* background, int width, int height, const float* means3D,
                              const float* shs, const float* colors_precomp, const float* opacities,
                              const float* scales, float scale_modifier, const float* rotations,
                              const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                              const float* cam_pos, float tan_fovx, float tan_fovy, int prefiltered, int foveaStep,
                              const float* out_color_precomp, char* geom_buffer_precomp,
                              char* binning_buffer_precomp, char* image_buffer_precomp, float* out_color, int* radii,
                              int interpolate_image, int debug, void* stream) {
    return gs_amr_rasterizer_forward_ex(geometry, binning, image, P, D, M, background, width, height, means3D, shs,
                                        colors_precomp, opacities, scales, scale_modifier, rotations, cov3D_precomp,
                                        viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered, foveaStep,
                                        out_color_precomp, geom_buffer_precomp, binning_buffer_precomp,
                                        image_buffer_precomp, out_color, radii, interpolate_image, debug, -1, stream);
}

int gs_amr_rasterizer_forward_ex(gs_buffer geometry, gs_buffer binning, gs_buffer image, int P, int D, int M,
                                 const float* background, int width, int height, const float* means3D,
                                 const float* shs, const float* colors_precomp, const float* opacities,
                                 const float* scales, float scale_modifier, const float* rotations,
                                 const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                                 const float* cam_pos, float tan_fovx, float tan_fovy, int prefiltered,
                                 int foveaStep, const float* out_color_precomp, char* geom_buffer_precomp,
                                 char* binning_buffer_precomp, char* image_buffer_precomp, float* out_color,
                                 int* radii, int interpolate_image, int debug, int num_rendered_hint, void* stream) {
    t_store_drgb = !take_fwd_no_grad();
    const bool step0_unfilled = t_amr_step0_unfilled != 0;  // (one-shot, consumed by every AMR forward)
    t_amr_step0_unfilled = 0;
    return guarded([&]() -> int {
        if (P <= 0) return 0;
        hipStream_t s = static_cast<hipStream_t>(stream);
        const int tile = 32;
        const int W = width, H = height;
        const int T = ((W + tile - 1) / tile) * ((H + tile - 1) / tile);
        const bool dbg = debug != 0;
        if (foveaStep >= 1) {
            // amr/cr/rasterizer_impl.cu:334-462: progressive step on precomputed buffers.
            if (!geom_buffer_precomp || !image_buffer_precomp)
                throw GsError("foveaStep >= 1 needs the buffers returned by foveaStep 0");
            GeomView g;
            ImageView img;
            BinningView b;
            carve_geom(geom_buffer_precomp, P, &g);
            carve_image(image_buffer_precomp, (size_t)W * H, T, &img, 32);
            int K = num_rendered_hint;
            if (K < 0) {  // the reference reads K back here (amr/cr/rasterizer_impl.cu:337-340)
                uint32_t hdr[4];
                read_header(g.hdr, hdr, s);
                K = (int)hdr[kHdrNumRendered];
            }
            if (K > 0 && !binning_buffer_precomp)
                throw GsError("foveaStep >= 1 needs the binning buffer returned by foveaStep 0");
            AmrBinningView ab;
            carve_binning(binning_buffer_precomp, K, &b, &ab);
            // variant 4 folds the step's level update and zero radii into its
            // render launch, and writes the zeros of the pixels it does not render
            const bool fused = g_amr_variant == 4;
            if (!fused) {
                launch_fovea_levels(foveaStep, T, img, s, P, radii);  // + the step's zero radii
                stage_check(dbg, s, "fovea_levels");
                GS_HIP(hipMemsetAsync(out_color, 0, sizeof(float) * 3 * (size_t)W * H, s));
            }
            const float* feats = colors_precomp ? colors_precomp : g.rgb;
            { StageTimer _t(kAmrRender, s);
              launch_amr_render(W, H, img, fused ? img.levels : img.levels_current, img.levels_last, b, ab, g, feats,
                                background, out_color, foveaStep, s, fused, P, radii); }
            stage_check(dbg, s, "amr_render");
            if (interpolate_image) {
                if (!out_color_precomp) throw GsError("interpolate_image at foveaStep >= 1 needs out_color_precomp");
                launch_amr_interpolate(W, H, img, img.levels_current, img.levels_last, out_color, foveaStep,
                                       out_color_precomp, s);
                stage_check(dbg, s, "amr_interpolate");
            }
            return K;
        }
        ForwardIn in{P, D, M, background, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                     viewmatrix, projmatrix, cam_pos, width, height, scale_modifier, tan_fovx, tan_fovy, prefiltered};
        // Everything that needs the tile counts / ranges but not K runs behind
        // the K copy, while the host waits for it: the levels (percentiles of
        // the counts), the step's level schedule, the tile order (by list
        // length) and step 0's zero image.
        auto before_k = [&](Binned& r) {
            // (variant 4 writes the zeros of the pixels it does not render;
            // otherwise, and at foveaStep 0, the levels launch zeroes the image)
            const bool zero_img = (foveaStep == 0 && !step0_unfilled) || g_amr_variant != 4;
            { StageTimer _t(kAmrLevels, s);
              launch_amr_levels(r.T, r.img, s, zero_img ? out_color : nullptr, zero_img ? 3 * (size_t)W * H : 0); }
            stage_check(dbg, s, "amr_levels");
            if (g_amr_variant == 4) launch_order_tiles(r.T, r.img, false, s);
            if (foveaStep != 0) launch_fovea_levels(foveaStep, r.T, r.img, s);
        };
        // the region-list pass sorts the tiles of <= kAmrFusedSortMax instances itself
        const bool fuse = g_amr_variant == 4 && fused_sort_on();
        Binned r = preprocess_and_bin(in, geometry, binning, image, radii, tile, dbg, s, before_k,
                                      fuse ? kAmrFusedSortMax : 0);
        // (the geometry buffer's own copy of the radii -- the progressive steps
        // return zero radii as the reference does, and the AMR backward of a
        // step reads the step-0 radii from there -- is written by the preprocess)
        const float* feats = colors_precomp ? colors_precomp : r.g.rgb;
        if (g_amr_variant == 4) {
            // the AMR blend's work units: tiles heaviest first (ordered above)
            // and their sub-lists: the 8x8 regions + blend records of the AMR
            // binning layout
            { StageTimer _t(kAmrLists, s); launch_amr_region_lists(W, H, r.img, r.b, r.ab, r.g, feats, r.K, s, fuse); }
            stage_check(dbg, s, "amr_lists");
        }
        if (foveaStep == 0) return r.K;  // step 0: buffers only, a zero image (amr/cr/rasterizer_impl.cu:651)
        { StageTimer _t(kAmrRender, s);
          launch_amr_render(W, H, r.img, r.img.levels, r.img.levels_last, r.b, r.ab, r.g, feats, background,
                            out_color, foveaStep, s); }
        stage_check(dbg, s, "amr_render");
        if (interpolate_image) {
            launch_amr_interpolate(W, H, r.img, r.img.levels, r.img.levels_last, out_color, foveaStep,
                                   out_color_precomp ? out_color_precomp : out_color, s);
            stage_check(dbg, s, "amr_interpolate");
        }
        return r.K;
    });
}

int gs_amr_accumulate_step(int P, const float* background, int width, int height, const float* colors_precomp,
                           int foveaStep, char* geom_buffer_precomp, char* binning_buffer_precomp,
                           char* image_buffer_precomp, float* accum, int* radii, int debug, int num_rendered_hint,
                           void* stream) {
    return guarded([&]() -> int {
        if (P <= 0) return 0;
        if ((foveaStep < 1 || foveaStep > 4) && foveaStep != kAmrStepsAll && foveaStep != kAmrStepsAllFill &&
            foveaStep != kAmrStepsAllSplit)
            throw GsError("gs_amr_accumulate_step: foveaStep in 1..4 or GSPLAT_AMD_AMR_STEPS_1_TO_4(_FILL, _SPLIT)");
        // _FILL: the same launch storing every pixel (0 + value, zeros where
        // nothing renders) instead of adding: accum holds an unfilled step-0 image.
        // _SPLIT: storing into the four steps' own images (accum [4][3][H][W],
        // radii [4][P])
        const bool fill = foveaStep == kAmrStepsAllFill, split = foveaStep == kAmrStepsAllSplit;
        if (fill || split) foveaStep = kAmrStepsAll;
        if (g_amr_variant != 4) throw GsError("gs_amr_accumulate_step needs the default amr_variant (4)");
        if (!geom_buffer_precomp || !image_buffer_precomp || !accum)
            throw GsError("gs_amr_accumulate_step needs the buffers returned by foveaStep 0 and the running image");
        hipStream_t s = static_cast<hipStream_t>(stream);
        const int W = width, H = height;
        const int T = ((W + 31) / 32) * ((H + 31) / 32);
        GeomView g;
        ImageView img;
        BinningView b;
        carve_geom(geom_buffer_precomp, P, &g);
        carve_image(image_buffer_precomp, (size_t)W * H, T, &img, 32);
        int K = num_rendered_hint;
        if (K < 0) {
            uint32_t hdr[4];
            read_header(g.hdr, hdr, s);
            K = (int)hdr[kHdrNumRendered];
        }
        if (K > 0 && !binning_buffer_precomp)
            throw GsError("gs_amr_accumulate_step needs the binning buffer returned by foveaStep 0");
        AmrBinningView ab;
        carve_binning(binning_buffer_precomp, K, &b, &ab);
        const float* feats = colors_precomp ? colors_precomp : g.rgb;
        { StageTimer _t(kAmrRender, s);
          launch_amr_render(W, H, img, img.levels, img.levels_last, b, ab, g, feats, background, accum, foveaStep, s,
                            true, split ? 4 * P : P, radii, split ? 2 : fill ? 0 : 1); }
        stage_check(debug != 0, s, "amr_render (accumulate)");
        return K;
    });
}

int gs_amr_set_step_state(char* image_buffer, size_t image_buffer_bytes, int width, int height, int step,
                          void* stream) {
    return guarded([&]() -> int {
        if (step < 1 || step > 4) throw GsError("gs_amr_set_step_state: step in 1..4");
        if (width <= 0 || height <= 0) return 0;
        if (!image_buffer) throw GsError("gs_amr_set_step_state: needs the image buffer of foveaStep 0");
        const size_t T = (size_t)((width + 31) / 32) * ((height + 31) / 32);
        if (image_buffer_bytes < carve_image(nullptr, (size_t)width * height, T, nullptr, 32))
            throw GsError("gs_amr_set_step_state: image buffer too small for width x height");
        ImageView img;
        carve_image(image_buffer, (size_t)width * height, T, &img, 32);
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_fovea_levels(kAmrStateAfter + step, (int)T, img, s);
        stage_check(false, s, "amr_set_step_state");
        return 0;
    });
}

int gs_amr_fovea_levels(char* image_buffer, size_t image_buffer_bytes, int width, int height, int nfovea, const float* centres_xy,
                        const float* radii, int min_level, int replace, void* stream) {
    return guarded([&]() -> int {
        if (nfovea < 0 || nfovea > 4) throw GsError("gs_amr_fovea_levels: 0 to 4 foveae");
        if (min_level < 0 || min_level > 4) throw GsError("gs_amr_fovea_levels: min_level in 0..4");
        if (width <= 0 || height <= 0) return 0;
        if (!image_buffer) throw GsError("gs_amr_fovea_levels: needs the image buffer of foveaStep 0");
        float cx[4], cy[4], r[4];
        for (int k = 0; k < nfovea; k++) {
            cx[k] = centres_xy[2 * k];
            cy[k] = centres_xy[2 * k + 1];
            r[k] = radii[k];
            if (!(r[k] >= 0.f)) throw GsError("gs_amr_fovea_levels: radii must be >= 0");
        }
        const int tile = 32;
        const size_t T = (size_t)((width + tile - 1) / tile) * ((height + tile - 1) / tile);
        if (image_buffer_bytes < carve_image(nullptr, (size_t)width * height, T, nullptr, tile))
            throw GsError("gs_amr_fovea_levels: image buffer too small for width x height");
        ImageView img;
        carve_image(image_buffer, (size_t)width * height, T, &img, tile);
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_fovea_override(width, height, img, nfovea, cx, cy, r, min_level, replace, s);
        stage_check(false, s, "amr_fovea_levels");
        return 0;
    });
}

int gs_simple_knn(int P, const float* points, float* mean_dists, gs_buffer scratch, void* stream) {
    return guarded([&]() -> int {
        if (P <= 0) return 0;
        char* ws = call_resize(scratch, knn_workspace_bytes(P), "knn scratch");
        { StageTimer _t(kKnn, static_cast<hipStream_t>(stream)); launch_knn(P, points, mean_dists, ws, static_cast<hipStream_t>(stream)); }
        stage_check(false, static_cast<hipStream_t>(stream), "knn");
        return 0;
    });
}

int gs_l1_ssim_loss(const float* image, const float* gt, int C, int H, int W, float lambda_dssim, float* grad,
                    float* out3, gs_buffer workspace, void* stream) {
    return guarded([&]() -> int {
        if (C <= 0 || H <= 0 || W <= 0) return 0;
        hipStream_t s = static_cast<hipStream_t>(stream);
        char* ws = call_resize(workspace, l1_ssim_workspace_bytes(C, H, W), "loss workspace");
        launch_l1_ssim(image, gt, C, H, W, lambda_dssim, grad, out3, reinterpret_cast<float*>(ws), s);
        stage_check(false, s, "l1_ssim");
        return 0;
    });
}

int gs_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, long long n, int nseg,
                 const long long* seg_end, const double* lr, const long long* step, double beta1, double beta2, double eps,
                 void* stream) {
    return guarded([&]() -> int {
        if (nseg < 1 || nseg > 8) throw GsError("gs_adam_step: 1..8 segments");
        for (int i = 0; i < nseg; i++)
            if (step[i] < 0 || (i > 0 && seg_end[i] < seg_end[i - 1])) throw GsError("gs_adam_step: bad segments");
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_adam(params, grads, exp_avg, exp_avg_sq, n, nseg, seg_end, lr, step, beta1, beta2, eps, s);
        stage_check(false, s, "adam");
        return 0;
    });
}

int gs_densify_stats(int P, const int* radii, const float* grad_means2D, int grad_stride, float* xyz_gradient_accum,
                     float* denom, float* max_radii2D, void* stream) {
    return guarded([&]() -> int {
        if (P < 0 || grad_stride < 2) throw GsError("gs_densify_stats: bad sizes");
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_densify_stats(P, radii, grad_means2D, grad_stride, xyz_gradient_accum, denom, max_radii2D, s);
        stage_check(false, s, "densify_stats");
        return 0;
    });
}

int gs_activate_gaussians(int P, int M, const float* features_dc, const float* features_rest, const float* opacity_raw,
                          const float* scaling_raw, const float* rotation_raw, float* shs, float* opacities,
                          float* scales, float* rotations, void* stream) {
    return guarded([&]() -> int {
        if (P < 0 || M < 1 || M > 16) throw GsError("gs_activate_gaussians: bad sizes");
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_activate(P, M, features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw, shs, opacities,
                        scales, rotations, s);
        stage_check(false, s, "activate");
        return 0;
    });
}

int gs_activation_backward(int P, int M, int accumulate, const float* dL_dshs, const float* dL_dopacities,
                           const float* dL_dscales, const float* dL_drotations, const float* dL_dmeans3D,
                           const float* opacity_raw, const float* scaling_raw, const float* rotation_raw,
                           float* grad_xyz, float* grad_features_dc, float* grad_features_rest, float* grad_opacity,
                           float* grad_scaling, float* grad_rotation, void* stream) {
    return guarded([&]() -> int {
        if (P < 0 || M < 1 || M > 16) throw GsError("gs_activation_backward: bad sizes");
        hipStream_t s = static_cast<hipStream_t>(stream);
        launch_activation_backward(P, M, accumulate, dL_dshs, dL_dopacities, dL_dscales, dL_drotations, dL_dmeans3D,
                                   opacity_raw, scaling_raw, rotation_raw, grad_xyz, grad_features_dc,
                                   grad_features_rest, grad_opacity, grad_scaling, grad_rotation, s);
        stage_check(false, s, "activation_backward");
        return 0;
    });
}

// Process-wide performance choices, each the default or one fallback; every
// pair produces the same results (bit-identical buffers, sums equal to
// atomic-order noise), so they are safe to flip between calls.
int gs_set_tuning(const char* key, int value) {
    if (!key) return -1;
    if (std::strcmp(key, "fwd_variant") == 0) {  // 0: one wave x 4 px predicate form; else the default
        set_forward_variant(value);
        return 0;
    }
    if (std::strcmp(key, "bwd_variant") == 0) {  // 0: predicate form, LDS-row sums; else the default (opacity-scaled sums)
        set_backward_variant(value);
        return 0;
    }
    if (std::strcmp(key, "amr_variant") == 0) {  // 0: full-list AMR blocks; else region sub-lists (default)
        set_amr_variant(value);
        return 0;
    }
    if (std::strcmp(key, "sort_algo") == 0) {  // 0: bitonic networks only; 1: per-tile bucket sort (default)
        set_sort_algo(value);
        return 0;
    }
    if (std::strcmp(key, "cull") == 0) {  // 0: no row-group cull in the blends (the exactness A/B)
        set_cull(value);
        return 0;
    }
    if (std::strcmp(key, "hdr_mirror") == 0) {  // 2: polled K read-back (default); 0: copy + event
        g_hdr_mirror = value == 0 ? 0 : 2;
        return 0;
    }
    if (std::strcmp(key, "spec_dup") == 0) {  // speculative duplicate before the K read-back (base forward)
        g_spec_dup = value;
        return 0;
    }
    if (std::strcmp(key, "ritnet_mfma") == 0) {  // 0: the SGPR-weight FMA convolution; 1: matrix cores (default)
        set_ritnet_mfma(value);
        return 0;
    }
    g_err = std::string("unknown tuning key ") + key;
    return -1;
}

// The current value of a gs_set_tuning key (the variants as they are used:
// 0 = the fallback, else the default's number).
int gs_get_tuning(const char* key, int* value) {
    if (!key || !value) return -1;
    hdr_mirror_on();  // (resolves the GSAMD_HDR_MIRROR default)
    const struct { const char* k; const int* v; } table[] = {
        {"fwd_variant", &g_fwd_variant}, {"bwd_variant", &g_bwd_variant}, {"amr_variant", &g_amr_variant},
        {"sort_algo", &g_sort_algo},     {"cull", &g_cull},               {"hdr_mirror", &g_hdr_mirror},
        {"spec_dup", &g_spec_dup},       {"ritnet_mfma", &g_ritnet_mfma}};
    for (const auto& e : table)
        if (std::strcmp(key, e.k) == 0) {
            *value = *e.v;
            return 0;
        }
    g_err = std::string("unknown tuning key ") + key;
    return -1;
}

int gs_set_thread_option(const char* key, int value) {
    if (!key) return -1;
    if (std::strcmp(key, "fwd_no_grad") == 0) {
        t_fwd_no_grad = value;
        return 0;
    }
    if (std::strcmp(key, "sh_drgb") == 0) {
        t_sh_drgb = value;
        return 0;
    }
    if (std::strcmp(key, "store_cov3d") == 0) {
        t_store_cov3d = value;
        return 0;
    }
    if (std::strcmp(key, "fwd_zero") == 0) {
        t_fwd_zero = value;
        return 0;
    }
    if (std::strcmp(key, "amr_step0_unfilled") == 0) {
        t_amr_step0_unfilled = value;
        return 0;
    }
    g_err = std::string("unknown thread option ") + key;
    return -1;
}

void gs_profile_enable(int on) {
    std::lock_guard<std::mutex> l(g_prof_mu);
    g_prof.on = on != 0;
}

void gs_profile_set_mask(unsigned mask) {
    std::lock_guard<std::mutex> l(g_prof_mu);
    g_prof.mask = mask;
}

int gs_profile_stage_count(void) { return kStages; }

const char* gs_profile_stage_name(int i) { return (i >= 0 && i < kStages) ? kStageNames[i] : ""; }

void gs_profile_read(double* total_ms, long* counts, int reset) {
    std::lock_guard<std::mutex> l(g_prof_mu);
    g_prof.harvest();
    for (int i = 0; i < kStages; i++) {
        if (total_ms) total_ms[i] = g_prof.total_ms[i];
        if (counts) counts[i] = g_prof.count[i];
        if (reset) {
            g_prof.total_ms[i] = 0;
            g_prof.count[i] = 0;
        }
    }
}

size_t gs_geom_bytes(int P) { return carve_geom(nullptr, (size_t)P, nullptr); }

size_t gs_amr_geom_bytes(int P) { return carve_geom(nullptr, (size_t)P, nullptr, true, true); }

size_t gs_image_bytes(int width, int height, int tile) {
    const size_t T = (size_t)((width + tile - 1) / tile) * ((height + tile - 1) / tile);
    return carve_image(nullptr, (size_t)width * height, T, nullptr, tile);
}

size_t gs_binning_bytes(int K) { return carve_binning(nullptr, (size_t)K, nullptr); }

namespace {
int binning_count_of_bytes(size_t nbytes, bool amr) {
    long lo = 0, hi = (long)std::min<size_t>(nbytes / 8 + 1, (size_t)INT32_MAX);
    while (lo < hi) {  // smallest K with bytes(K) >= nbytes (bytes() is strictly increasing)
        const long mid = (lo + hi) / 2;
        if (carve_binning(nullptr, (size_t)mid, nullptr, nullptr, amr) < nbytes) lo = mid + 1;
        else hi = mid;
    }
    return carve_binning(nullptr, (size_t)lo, nullptr, nullptr, amr) == nbytes ? (int)lo : -1;
}
}  // namespace

int gs_binning_count_of_bytes(size_t nbytes) { return binning_count_of_bytes(nbytes, false); }

size_t gs_amr_binning_bytes(int K) { return carve_binning(nullptr, (size_t)K, nullptr, nullptr, true); }

int gs_amr_binning_count_of_bytes(size_t nbytes) { return binning_count_of_bytes(nbytes, true); }

size_t gs_knn_workspace_bytes(int P) { return knn_workspace_bytes(P); }

int gs_geom_view_of(char* base, int P, gs_geom_view* out) {
    GeomView g;
    carve_geom(base, (size_t)P, &g);
    static_assert(sizeof(GeomView) == sizeof(gs_geom_view), "view layout");
    std::memcpy(out, &g, sizeof(g));
    return 0;
}

int gs_image_view_of(char* base, int width, int height, int tile, gs_image_view* out) {
    const size_t T = (size_t)((width + tile - 1) / tile) * ((height + tile - 1) / tile);
    ImageView v;
    carve_image(base, (size_t)width * height, T, &v, tile);
    static_assert(sizeof(ImageView) == sizeof(gs_image_view), "view layout");
    std::memcpy(out, &v, sizeof(v));
    return 0;
}

int gs_binning_view_of(char* base, int K, gs_binning_view* out) {
    BinningView v;
    carve_binning(base, (size_t)K, &v);
    static_assert(sizeof(BinningView) == sizeof(gs_binning_view), "view layout");
    std::memcpy(out, &v, sizeof(v));
    return 0;
}

int gs_reconstruct_keys(char* geom_buffer, char* binning_buffer, char* img_buffer, int P, int K, int width,
                        int height, int tile, uint64_t* keys_out, void* stream) {
    return guarded([&]() -> int {
        const int T = ((width + tile - 1) / tile) * ((height + tile - 1) / tile);
        GeomView g;
        ImageView img;
        BinningView b;
        carve_geom(geom_buffer, P, &g);
        carve_image(img_buffer, (size_t)width * height, T, &img, tile);
        carve_binning(binning_buffer, K, &b);
        if (K > 0) launch_reconstruct_keys(T, img, b, g, keys_out, static_cast<hipStream_t>(stream));
        stage_check(false, static_cast<hipStream_t>(stream), "reconstruct_keys");
        return 0;
    });
}

}  // extern "C"
