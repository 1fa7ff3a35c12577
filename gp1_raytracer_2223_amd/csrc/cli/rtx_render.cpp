// rtx_render — headless C++ host program (the reference's main.cpp frame loop without
// the SDL window): builds a catalogue scene with librtx_host.so, renders it through the
// C-ABI of librtx_hip.so and writes RayTracing_Buffer.bmp like the reference's X key.
//
//   rtx_render <scene> [width height] [--time T] [--mode 0..3] [--no-shadows]
//              [--frames N] [--out file.bmp] [--assets dir] [--benchmark [windows]] [--inflight F]
//              [--device-update]
//
// --benchmark runs the reference's frame loop (main.cpp:86-100: Scene::Update with the
// timer's total time, Render into the host pixel buffer, Timer::Update) under its F6
// benchmark (Timer.cpp:44-131): `windows` one-second dFPS windows (default 10), then
// ">> HIGH/LOW/AVG" on stdout and benchmark.txt in the reference's format.  Animated
// scenes are re-uploaded after every Update; the per-stage means are printed as well.
// --inflight F (default 2) overlaps F frames (run_benchmark); 1 = the serial loop.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include <sys/resource.h>

#include "benchmark.h"
#include "rtx_renderer.hpp"

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }
double cpu_secs() {   // the process's CPU time, every thread (user + system)
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return double(u.ru_utime.tv_sec + u.ru_stime.tv_sec) + 1e-6 * double(u.ru_utime.tv_usec + u.ru_stime.tv_usec);
}

// The pipelined host side of run_benchmark.  The reference's BuildBVH permutes the triangles in
// place (DataTypes.h:335-363), so the state Update k leaves depends on every earlier Update: ONE
// chain scene is updated serially, on a worker thread, and after Update k its state is copied into
// snapshot k % D (rtx_host_scene_copy_state), which the main thread uploads.  The worker runs up to D
// frames ahead of the uploads: Update k + 1 overlaps frame k's upload and the GPU's frames, and only
// the snapshot copy waits for its slot.  time_of(k) gives frame k's Update time (taken when that
// Update starts); `limit` (>= 0) stops the worker after that many frames.
class ChainUpdater {
public:
    ChainUpdater(rtx_host_scene* chain, std::vector<rtx_host_scene*> snaps, std::function<float(long)> time_of,
                 long limit)
        : chain_(chain), snaps_(std::move(snaps)), time_of_(std::move(time_of)), limit_(limit),
          th_([this] { Loop(); }) {}
    ~ChainUpdater() {
        {
            std::lock_guard<std::mutex> l(m_);
            quit_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // frame k's snapshot, once Update k has been copied into it (nullptr if the worker failed)
    rtx_host_scene* wait(long k) {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return ready_ > k || failed_; });
        return failed_ ? nullptr : snaps_[k % snaps_.size()];
    }
    // frame k's upload has returned (the upload copied the arrays): its snapshot may be overwritten
    void release(long k) {
        std::lock_guard<std::mutex> l(m_);
        released_ = std::max(released_, k + 1);
        cv_.notify_all();
    }

private:
    void Loop() {
        const long D = static_cast<long>(snaps_.size());
        for (long k = 0;; ++k) {
            {
                std::lock_guard<std::mutex> l(m_);
                if (quit_ || (limit_ >= 0 && k >= limit_)) return;
            }
            rtx_host_scene_update(chain_, time_of_(k));   // Scene::Update, in the reference's order
            std::unique_lock<std::mutex> l(m_);
            cv_.wait(l, [&] { return quit_ || k < released_ + D; });
            if (quit_) return;
            l.unlock();
            const int rc = rtx_host_scene_copy_state(snaps_[k % D], chain_);
            l.lock();
            if (rc != RTX_OK) failed_ = true;
            ready_ = k + 1;
            cv_.notify_all();
            if (failed_) return;
        }
    }
    rtx_host_scene* chain_;
    std::vector<rtx_host_scene*> snaps_;
    std::function<float(long)> time_of_;
    long limit_;
    std::mutex m_;
    std::condition_variable cv_;
    long ready_ = 0, released_ = 0;
    bool quit_ = false, failed_ = false;
    std::thread th_;   // (last: started after the members above)
};

// The reference's frame loop is serial: Update, Render (into the window surface), present.
// Here `inflight` frames overlap: frame k is updated, uploaded and queued (render + D2H into
// its own page-locked host frame) on context k % inflight while frame k - 1 still runs on
// another context's stream, so the host's Update / BVH rebuild of the next frame hides
// behind the current frame's GPU work.  Every frame is still fully rendered and in host
// memory before it counts: the benchmark ticks when frame k's context has finished.
// inflight = 1 is the reference's serial loop.
// With frames in flight and more host scenes of the same catalogue scene (`extra`, D of them) the
// host side is pipelined too (ChainUpdater): `hs` is updated serially on a worker thread, one
// Update history as in the reference's loop, and each frame's state is uploaded from a snapshot
// (one of the D extra scenes) while the worker goes on with the next Updates (an upload copies the
// host arrays into page-locked staging before it returns, so the snapshot is free again after it).
// A frame's time is taken when its Update starts.
// --device-update: the animated meshes' Update (transform + BVH rebuild + scene image) runs on
// the device (rtx_anim_*); the host only computes the frame's transforms.
// With `seq` (--sequence t1,t2,...): no timer; frame k is Update(seq[k]) and is written to
// `<stem>_<k>.bmp` when it completes (the pipelined loop's frames, checked by the tests).
int run_benchmark(rtx::Renderer& r, rtx_host_scene* hs, int windows, int inflight, bool device_update,
                  const std::vector<float>* seq = nullptr, const std::string& stem = "",
                  const std::vector<rtx_host_scene*>& extra = {}) {
    const bool animated = rtx_host_scene_animated(hs) == 1;
    // (pipelined host side) D = the snapshot scenes: `hs` is the chain the worker updates, frame k is
    // uploaded from snapshot extra[k % D]
    const int D = (animated && !device_update && inflight >= 2) ? static_cast<int>(extra.size()) : 0;
    const bool pipe = D > 0;
    const size_t npx = static_cast<size_t>(r.Width()) * r.Height();
    std::vector<rtx_ctx*> ctx{r.Context()};
    for (int f = 1; f < inflight; ++f) {
        rtx_ctx* c = nullptr;
        if (rtx_create(&c, 0) != RTX_OK) {
            std::fprintf(stderr, "rtx_create: %s\n", rtx_last_error(nullptr));
            for (size_t i = 1; i < ctx.size(); ++i) rtx_destroy(ctx[i]);
            return 1;
        }
        ctx.push_back(c);
    }
    std::vector<std::vector<uint32_t>> buf(inflight, std::vector<uint32_t>(npx));
    std::vector<char> upd_ok(inflight, 1);   // --sequence: the device Update of the frame in buf[f] succeeded
    for (int f = 0; f < inflight; ++f) rtx_host_register(ctx[f], buf[f].data(), npx * 4);   // async D2H
    const rtx_render_params p = r.Params();
    rtx::Benchmark b(windows);
    if (!seq) std::cout << "**BENCHMARK STARTED**\n";
    double t_update = 0, t_upload = 0, t_queue = 0, t_wait = 0;
    long frames = 0, queued = 0;
    int rc = 0, last = -1;
    const Clock::time_point start = Clock::now();
    const double cpu0 = cpu_secs();
    Clock::time_point prev = start;
    std::unique_ptr<ChainUpdater> chain;
    if (pipe)
        chain.reset(new ChainUpdater(
            hs, extra, [&](long k) { return seq ? (*seq)[k] : static_cast<float>(secs(start, Clock::now())); },
            seq ? static_cast<long>(seq->size()) : -1));
    rtx_scene s;
    rtx_camera cam;
    auto ok = [&](int code, const char* what, rtx_ctx* c) {
        if (code == RTX_OK) return true;
        std::fprintf(stderr, "%s: %s\n", what, rtx_last_error(c));
        rc = 1;
        return false;
    };
    // device-side Update: register the scene's turning meshes on the first context
    rtx_anim* anim = nullptr;
    std::vector<float> mats;
    int n_anim = 0;
    // every registered mesh's device Update status (NaN vertex, a tree too deep to render)
    auto anim_ok = [&]() {
        for (int i = 0; i < n_anim; ++i) {
            uint32_t st[4];
            if (rtx_anim_status(anim, static_cast<uint32_t>(i), st) != RTX_OK) {
                std::fprintf(stderr, "device Update failed (registered mesh %d): %s\n", i, rtx_anim_last_error(anim));
                return false;
            }
        }
        return true;
    };
    if (device_update && animated) {
        std::vector<int32_t> ids(64);
        const int ns = rtx_host_scene_spinning(hs, ids.data(), static_cast<uint32_t>(ids.size()));
        if (ns > static_cast<int>(ids.size())) {   // rtx_anim_create takes at most 32 anyway
            std::fprintf(stderr, "--device-update: %d turning meshes, more than %zu\n", ns, ids.size());
            for (size_t i = 1; i < ctx.size(); ++i) rtx_destroy(ctx[i]);
            return 1;
        }
        n_anim = ns;
        std::vector<rtx_mesh_source> src(ns > 0 ? ns : 0);
        for (int i = 0; i < ns; ++i) rtx_host_scene_mesh_source(hs, static_cast<uint32_t>(ids[i]), &src[i]);
        rtx_host_scene_view(hs, &s, &cam);
        if (ns <= 0 || rtx_anim_create(&anim, ctx[0], &s, ids.data(), src.data(), static_cast<uint32_t>(ns)) != RTX_OK) {
            std::fprintf(stderr, "rtx_anim_create: %s\n", rtx_anim_last_error(nullptr));
            for (size_t i = 1; i < ctx.size(); ++i) rtx_destroy(ctx[i]);
            return 1;
        }
        mats.resize(16 * static_cast<size_t>(ns));
    }
    for (;;) {
        const int f = static_cast<int>(queued % inflight);
        if (queued >= inflight) {   // frame queued - inflight (this context's) completes
            const Clock::time_point w0 = Clock::now();
            if (!ok(rtx_synchronize(ctx[f]), "rtx_synchronize", ctx[f])) break;
            const Clock::time_point w1 = Clock::now();
            t_wait += secs(w0, w1);
            ++frames;
            last = f;
            const float elapsed = static_cast<float>(secs(prev, w1));                  // Timer::Update
            prev = w1;
            if (seq) {
                if (anim && !upd_ok[f]) { rc = 1; break; }   // never write a frame of a failed Update
                r.Pixels() = buf[f];
                if (!r.SaveBufferToImage(stem + "_" + std::to_string(frames - 1) + ".bmp")) { rc = 1; break; }
                if (frames == static_cast<long>(seq->size())) break;
            } else if (b.Tick(elapsed)) {
                break;
            }
        }
        if (seq && queued >= static_cast<long>(seq->size())) {   // drain: nothing left to queue
            ++queued;
            continue;
        }
        const Clock::time_point f0 = Clock::now();
        const float tnow = seq ? (*seq)[queued] : static_cast<float>(secs(start, f0));
        rtx_host_scene* cur = hs;
        if (pipe) {
            cur = chain->wait(queued);   // frame `queued`'s Update (the worker's chain), in its snapshot
            if (!cur) {
                std::fprintf(stderr, "rtx_host_scene_copy_state failed\n");
                rc = 1;
                break;
            }
        } else if (anim) {
            rtx_host_scene_transforms(hs, tnow, mats.data(), static_cast<uint32_t>(n_anim));   // Update(t)'s turn
        } else if (animated) {
            rtx_host_scene_update(hs, tnow);                // Scene::Update
        }
        const Clock::time_point f1 = Clock::now();
        if (!ok(rtx_host_scene_view(cur, &s, &cam), "rtx_host_scene_view", nullptr)) break;
        if (anim) {
            if (rtx_anim_update(anim, ctx[f], mats.data()) != RTX_OK) {
                std::fprintf(stderr, "rtx_anim_update: %s\n", rtx_anim_last_error(anim));
                rc = 1;
                break;
            }
            // --sequence: this Update's own status, read now (the status words are the newest
            // Update's, so with frames in flight a later one would overwrite a failure); the
            // frame is written only if it is clean.  The benchmark loop checks once at the end.
            if (seq) upd_ok[f] = anim_ok();
        } else if ((animated || queued < inflight) && !ok(rtx_upload_scene(ctx[f], &s), "rtx_upload_scene", ctx[f])) {
            break;
        }
        if (pipe) chain->release(queued);   // the upload copied the snapshot's arrays
        const Clock::time_point f2 = Clock::now();
        if (!ok(rtx_render_async(ctx[f], &cam, &p, 0), "rtx_render_async", ctx[f])) break;  // Renderer::Render
        if (!ok(rtx_gather_async(ctx[f], buf[f].data(), nullptr), "rtx_gather_async", ctx[f])) break;
        const Clock::time_point f3 = Clock::now();
        t_update += secs(f0, f1);
        t_upload += secs(f1, f2);
        t_queue += secs(f2, f3);
        ++queued;
    }
    for (int f = 0; f < inflight; ++f) rtx_synchronize(ctx[f]);
    chain.reset();   // (stops the worker after its current Update)
    if (anim) {
        if (!anim_ok()) rc = 1;
        rtx_anim_destroy(anim);
    }
    if (last >= 0) r.Pixels() = buf[last];   // the last completed frame (SaveBufferToImage)
    for (int f = 0; f < inflight; ++f) rtx_host_unregister(ctx[f], buf[f].data());
    for (size_t i = 1; i < ctx.size(); ++i) rtx_destroy(ctx[i]);
    if (rc || seq) return rc;
    rtx::WriteBenchmark(b);
    const double n = static_cast<double>(queued);
    // host CPU use of the loop: process CPU time (the build pool's spinning workers included) over
    // wall time, in cores
    const double cores = (cpu_secs() - cpu0) / std::max(1e-9, secs(start, Clock::now()));
    std::printf("frames %ld%s%s, %d in flight: per frame update %.3f ms, upload %.3f ms, queue %.3f ms, "
                "wait for GPU %.3f ms, host CPU %.2f cores\n", frames, animated ? " (animated)" : "",
                device_update ? " device Update" : "", inflight, t_update / n * 1e3,
                t_upload / n * 1e3, t_queue / n * 1e3, t_wait / std::max(1.0, double(frames)) * 1e3, cores);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene> [width height] [--time T] [--mode M] [--no-shadows] [--frames N] "
                             "[--out f.bmp] [--assets dir] [--benchmark [windows]] [--inflight F] [--device-update]\n",
                     argv[0]);
        return 2;
    }
    std::string scene = argv[1], out = "RayTracing_Buffer.bmp", assets;
    int W = 640, H = 480, mode = 3, frames = 1, bench = 0, inflight = 2;
    std::vector<float> seq;
    float t = -1.f;
    bool shadows = true, device_update = false;
    int pos = 0;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--time" && i + 1 < argc) t = std::strtof(argv[++i], nullptr);
        else if (a == "--mode" && i + 1 < argc) mode = std::atoi(argv[++i]);
        else if (a == "--no-shadows") shadows = false;
        else if (a == "--frames" && i + 1 < argc) frames = std::atoi(argv[++i]);
        else if (a == "--sequence" && i + 1 < argc) {
            for (const char* q = argv[++i]; *q;) {
                char* e = nullptr;
                seq.push_back(std::strtof(q, &e));
                q = (*e == ',') ? e + 1 : e;
                if (e == q && *q) break;
            }
        }
        else if (a == "--inflight" && i + 1 < argc) inflight = std::max(1, std::min(8, std::atoi(argv[++i])));
        else if (a == "--device-update") device_update = true;
        else if (a == "--out" && i + 1 < argc) out = argv[++i];
        else if (a == "--assets" && i + 1 < argc) assets = argv[++i];
        else if (a == "--benchmark") bench = (i + 1 < argc && std::atoi(argv[i + 1]) > 0) ? std::atoi(argv[++i]) : 10;
        else if (pos == 0) { W = std::atoi(argv[i]); ++pos; }
        else if (pos == 1) { H = std::atoi(argv[i]); ++pos; }
    }
    char err[512] = {0};
    rtx_host_scene* hs = nullptr;
    if (rtx_host_scene_create(scene.c_str(), assets.empty() ? nullptr : assets.c_str(), &hs, err, sizeof err) != RTX_OK) {
        std::fprintf(stderr, "scene %s: %s\n", scene.c_str(), err);
        return 1;
    }
    if (t >= 0.f) rtx_host_scene_update(hs, t);
    // the pipelined loop's second host scene (run_benchmark): animated scenes, frames in flight,
    // host Update
    // (up to two more: two Updates in flight with three or more frames in flight)
    auto more_scenes = [&]() {
        std::vector<rtx_host_scene*> v;
        if (inflight < 2 || device_update || rtx_host_scene_animated(hs) != 1) return v;
        for (int i = 0; i < std::min(inflight, 3) - 1; ++i) {
            rtx_host_scene* h = nullptr;
            char e2[512] = {0};
            if (rtx_host_scene_create(scene.c_str(), assets.empty() ? nullptr : assets.c_str(), &h, e2, sizeof e2) != RTX_OK)
                break;   // (fewer Updates in flight, or the loop unpipelined)
            v.push_back(h);
        }
        return v;
    };
    int rc = 0;
    try {
        rtx::Renderer r(W, H);
        r.m_CurrentLightingMode = static_cast<rtx::Renderer::LightingMode>(mode);
        r.m_ShadowsEnabled = shadows;
        if (!seq.empty()) {
            // --sequence t1,...: the pipelined frame loop over fixed Update times, frame k
            // written to <out stem>_<k>.bmp
            const std::string stem = out.size() > 4 && out.substr(out.size() - 4) == ".bmp" ? out.substr(0, out.size() - 4) : out;
            const std::vector<rtx_host_scene*> more = more_scenes();
            rc = run_benchmark(r, hs, 0, inflight, device_update, &seq, stem, more);
            for (rtx_host_scene* h : more) rtx_host_scene_destroy(h);
            rtx_host_scene_destroy(hs);
            return rc;
        }
        if (bench) {
            const std::vector<rtx_host_scene*> more = more_scenes();
            rc = run_benchmark(r, hs, bench, inflight, device_update, nullptr, "", more);
            for (rtx_host_scene* h : more) rtx_host_scene_destroy(h);
        } else {
            r.Render(hs, true);
            auto t0 = Clock::now();
            for (int f = 1; f < frames; ++f) r.Render(hs, false);
            auto t1 = Clock::now();
            if (frames > 1) {
                const double s = secs(t0, t1) / (frames - 1);
                std::printf("%s %dx%d: %.3f ms/frame incl. D2H, %.1f Mpix/s\n", scene.c_str(), W, H, s * 1e3,
                            W * (double)H / s / 1e6);
            }
        }
        if (rc == 0 && !r.SaveBufferToImage(out)) { std::fprintf(stderr, "cannot write %s\n", out.c_str()); rc = 1; }
        else if (rc == 0) std::printf("wrote %s\n", out.c_str());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        rc = 1;
    }
    rtx_host_scene_destroy(hs);
    return rc;
}
