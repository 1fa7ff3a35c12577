// rtx_group.cpp — one frame tiled across several render contexts (GPUs) by ONE host
// process: SURVEY §8(e)'s single-process driver.  Built into librtx_hip.so on top of the
// per-context C-ABI (rtx.h); no HIP call of its own.
//
// The reference renders a frame with concurrency::parallel_for over every pixel
// (source/Renderer.cpp:79-85): pixels are independent and there is no exchange step.
// Here the frame's rows are cut into `stripe_rows`-row stripes dealt round robin over the
// G members (member i owns stripes s with s % G == i: contiguous bands would load-
// imbalance around the mesh and its shadows).  Each member has a persistent host thread
// that renders its stripes on its own context stream (rtx_render_async) and queues the
// strided D2H copy straight into the caller's full-frame host buffer (rtx_gather_async:
// one hipMemcpy2DAsync per plane), then waits for its stream.  The caller's thread waits
// for all members: rtx_group_render is blocking, like Renderer::Render.  No collective,
// no peer traffic: each GPU's stripes cross its own PCIe link once.
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "rtx.h"

struct rtx_group {
    std::vector<rtx_ctx*> ctx;
    std::vector<std::thread> workers;
    std::mutex mu;
    std::condition_variable go, done;
    uint64_t gen = 0;   // job generation: a worker runs each new generation once
    int pending = 0;
    bool quit = false;
    // current job
    enum Op { kUpload, kRender } op = kUpload;
    const rtx_scene* scene = nullptr;
    const rtx_camera* cam = nullptr;
    rtx_render_params params{};
    uint32_t* out_px = nullptr;
    float* out_rgb = nullptr;
    std::vector<int> rc;
    std::string err;
};

namespace {

thread_local std::string g_group_create_err;

int run_member(rtx_group* g, size_t i) {
    rtx_ctx* c = g->ctx[i];
    if (g->op == rtx_group::kUpload) return rtx_upload_scene(c, g->scene);
    rtx_render_params p = g->params;
    const uint32_t n = static_cast<uint32_t>(g->ctx.size());
    if (n > 1) {
        p.stripe_rows = p.stripe_rows ? p.stripe_rows : 16u;
        p.stripe_first = static_cast<uint32_t>(i);
        p.stripe_step = n;
    } else {
        p.stripe_rows = 0;
        p.stripe_first = 0;
        p.stripe_step = 1;
    }
    int rc = rtx_render_async(c, g->cam, &p, g->out_rgb != nullptr);
    if (rc == RTX_OK) rc = rtx_gather_async(c, g->out_px, g->out_rgb);
    if (rc == RTX_OK) rc = rtx_synchronize(c);
    return rc;
}

void worker_loop(rtx_group* g, size_t i) {
    uint64_t seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(g->mu);
            g->go.wait(lk, [&] { return g->quit || g->gen != seen; });
            if (g->quit) return;
            seen = g->gen;
        }
        const int rc = run_member(g, i);
        std::lock_guard<std::mutex> lk(g->mu);
        g->rc[i] = rc;
        if (--g->pending == 0) g->done.notify_all();
    }
}

// Run the current job on every member and wait; the first failing member's error wins.
int run_job(rtx_group* g) {
    {
        std::lock_guard<std::mutex> lk(g->mu);
        std::fill(g->rc.begin(), g->rc.end(), RTX_OK);
        g->pending = static_cast<int>(g->ctx.size());
        ++g->gen;
    }
    g->go.notify_all();
    std::unique_lock<std::mutex> lk(g->mu);
    g->done.wait(lk, [&] { return g->pending == 0; });
    for (size_t i = 0; i < g->rc.size(); ++i) {
        if (g->rc[i] != RTX_OK) {
            g->err = "member " + std::to_string(i) + ": " + rtx_last_error(g->ctx[i]);
            return g->rc[i];
        }
    }
    g->err.clear();
    return RTX_OK;
}

}  // namespace

extern "C" int rtx_group_create(rtx_group** out, const int* device_ids, int n) {
    if (!out) return RTX_E_INVALID;
    *out = nullptr;
    g_group_create_err.clear();
    if (!device_ids || n < 1 || n > RTX_GROUP_MAX) {
        g_group_create_err = "need 1..RTX_GROUP_MAX device ids";
        return RTX_E_INVALID;
    }
    rtx_group* g = new (std::nothrow) rtx_group;
    if (!g) return RTX_E_NOMEM;
    for (int i = 0; i < n; ++i) {
        rtx_ctx* c = nullptr;
        const int rc = rtx_create(&c, device_ids[i]);
        if (rc != RTX_OK) {
            g_group_create_err = "device " + std::to_string(device_ids[i]) + ": " + rtx_last_error(nullptr);
            rtx_group_destroy(g);
            return rc;
        }
        g->ctx.push_back(c);
    }
    g->rc.assign(g->ctx.size(), RTX_OK);
    try {
        for (size_t i = 0; i < g->ctx.size(); ++i) g->workers.emplace_back(worker_loop, g, i);
    } catch (...) {
        g_group_create_err = "could not start the member threads";
        rtx_group_destroy(g);
        return RTX_E_NOMEM;
    }
    *out = g;
    return RTX_OK;
}

extern "C" void rtx_group_destroy(rtx_group* g) {
    if (!g) return;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->quit = true;
    }
    g->go.notify_all();
    for (auto& t : g->workers)
        if (t.joinable()) t.join();
    for (rtx_ctx* c : g->ctx) rtx_destroy(c);
    delete g;
}

extern "C" const char* rtx_group_last_error(const rtx_group* g) {
    return g ? g->err.c_str() : g_group_create_err.c_str();
}

extern "C" int rtx_group_size(const rtx_group* g) { return g ? static_cast<int>(g->ctx.size()) : 0; }

extern "C" rtx_ctx* rtx_group_context(rtx_group* g, int i) {
    if (!g || i < 0 || i >= static_cast<int>(g->ctx.size())) return nullptr;
    return g->ctx[static_cast<size_t>(i)];
}

extern "C" int rtx_group_upload_scene(rtx_group* g, const rtx_scene* s) {
    if (!g || !s) return RTX_E_INVALID;
    g->op = rtx_group::kUpload;
    g->scene = s;
    return run_job(g);
}

extern "C" int rtx_group_render(rtx_group* g, const rtx_camera* cam, const rtx_render_params* p, uint32_t* out_px,
                                float* out_rgb) {
    if (!g || !cam || !p || !out_px) return RTX_E_INVALID;
    if (p->stripe_step > 1) {
        g->err = "rtx_group_render partitions the frame itself: stripe_step must be 0 or 1";
        return RTX_E_INVALID;
    }
    if (p->stripe_rows % 16 != 0) {
        g->err = "stripe_rows must be a multiple of 16 (0 = 16)";
        return RTX_E_INVALID;
    }
    g->op = rtx_group::kRender;
    g->cam = cam;
    g->params = *p;
    g->out_px = out_px;
    g->out_rgb = out_rgb;
    return run_job(g);
}
