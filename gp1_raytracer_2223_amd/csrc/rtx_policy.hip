// rtx_policy.hip — the frame policies of the render context (rtx_ctx.h): which tiles a frame splits
// and how (the split tuner, throughput mode and the in-flight one-piece choice), the frontier
// refinement, and when the split chain joins the frame stream.  Host code only; no pixel depends on
// any of it (every choice renders the reference's frame).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "rtx_ctx.h"

namespace rtxh {

namespace {
// The process's contexts that have queued a frame (rtx_ctx::ev_frame), for throughput mode.
std::mutex g_frames_m;
std::vector<rtx_ctx*> g_frames;

}  // namespace

// The other contexts on c's device with a frame still in flight (their ev_frame not reached).
uint32_t frames_concurrent(rtx_ctx* c) {
    std::lock_guard<std::mutex> l(g_frames_m);
    uint32_t n = 0;
    for (rtx_ctx* o : g_frames) {
        if (o == c || o->device != c->device) continue;
        const hipError_t q = hipEventQuery(o->ev_frame);
        if (q == hipErrorNotReady) {
            (void)hipGetLastError();   // (not-ready is no error for the caller's checks)
            ++n;
        }
    }
    return n;
}
void frames_note(rtx_ctx* c) {
    std::lock_guard<std::mutex> l(g_frames_m);
    if (std::find(g_frames.begin(), g_frames.end(), c) == g_frames.end()) g_frames.push_back(c);
}
void frames_forget(rtx_ctx* c) {
    std::lock_guard<std::mutex> l(g_frames_m);
    g_frames.erase(std::remove(g_frames.begin(), g_frames.end(), c), g_frames.end());
}

// One step of the split-threshold tuner (rtx_ctx::tune_*): the timed frame rendered the heavy set
// selected with factor tune_rec_permille; main = its main kernel, chain = the split launches (both
// from the fork).  The next factor is a step away from THAT factor (a set selected with an older
// factor is not evidence about the current one), toward the balance of the two.
// The frame span max(main, chain) of every factor tried is kept: a step that makes it 5 % worse
// than the best seen returns to the best and stops (a GPU that cannot run the chain beside the main
// kernel — a profiler serialising dispatches, another process — would otherwise drift the factor).
void split_tune(rtx_ctx* c, float main_ms, float chain_ms) {
    const uint32_t base = c->tune_rec_permille;
    if (!base || main_ms <= 0.f || chain_ms <= 0.f) return;
    if (base != c->split_permille) return;   // a set from before the last step: wait for the current one
    const float span = std::max(main_ms, chain_ms);
    if (c->tune_best_permille == 0 || span < c->tune_best_span) {
        c->tune_best_span = span;
        c->tune_best_permille = base;
    } else if (span > 1.05f * c->tune_best_span) {
        c->split_permille = c->tune_best_permille;
        c->tune_done = true;
        return;
    }
    const float r = chain_ms / main_ms;
    const int dir = r > 1.04f ? 1 : (r < 0.96f ? -1 : 0);
    if (dir == 0 || ++c->tune_steps > 16) {
        c->tune_done = true;
        return;
    }
    if (c->tune_dir != 0 && dir != c->tune_dir) c->tune_step = std::sqrt(c->tune_step);   // overshot
    if (c->tune_step < 1.015f) {
        c->tune_done = true;
        return;
    }
    c->tune_dir = dir;
    const double f = static_cast<double>(base) * (dir > 0 ? c->tune_step : 1.0 / c->tune_step);
    c->split_permille = static_cast<uint32_t>(std::min(4000.0, std::max(1000.0, f)));
}

// Join the last frame's split chain into the frame stream (rtx_ctx::join_pending) before anything
// that reads its pixels, reallocates or rewrites what it reads, or needs the frame complete.
int join_split(rtx_ctx* c) {
    if (!c->join_pending) return RTX_OK;
    c->join_pending = false;
    HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
    return RTX_OK;
}

// One round of the frontier refinement (kRefineRounds), once the measured frame has completed
// (rtx_ctx::ev_refine; not waited for): per part the longest closest-hit wave plus the longest
// shadow wave; the parts within kRefineTopPermille of the longest are replaced by their two
// children (inner nodes only; the order of the frontier kept), and the new frontier is copied into
// the image's parts section on the frame stream, behind every frame already queued.
int refine_round(rtx_ctx* c) {
    const hipError_t q = hipEventQuery(c->ev_refine);
    (void)hipGetLastError();   // (not-ready is no error for the caller's checks)
    if (q == hipErrorNotReady) return RTX_OK;
    HIP_TRY(c, q);
    HIP_TRY(c, hipMemcpy(c->h_part_max.data(), c->d_part_max, c->h_part_max.size() * sizeof(uint32_t),
                         hipMemcpyDeviceToHost));
    const size_t np = c->h_parts.size();
    std::vector<uint64_t> m(np, 0);
    uint64_t top = 0;
    for (size_t p = 0; p < np; ++p) {
        uint32_t a = 0, b = 0;
        for (int k = 0; k < kPartShards; ++k) {
            a = std::max(a, c->h_part_max[(0 * kMaxParts + p) * kPartShards + k]);
            b = std::max(b, c->h_part_max[(1 * kMaxParts + p) * kPartShards + k]);
        }
        m[p] = static_cast<uint64_t>(a) + b;
        top = std::max(top, m[p]);
    }
    ++c->refine_round;
    // done: nothing measured, the last round gained under 10 %, or the rounds are spent
    const bool gained = c->refine_prev_max == 0 || top * 10 < static_cast<uint64_t>(c->refine_prev_max) * 9;
    c->refine_prev_max = static_cast<uint32_t>(std::min<uint64_t>(top, 0xffffffffull));
    c->refine_state = 2;
    if (top * kSplitMinUs < static_cast<uint64_t>(kRefineMinUs) * kSplitMinCost || !gained) return RTX_OK;
    // only a chain whose longest waves outlast the main kernel by kRefineOverMain: with less, the
    // frame is bound by its work (more parts only add waves; frames in flight lose throughput)
    const double top_ms = static_cast<double>(top) * kSplitMinUs / kSplitMinCost * 1e-3;
    if (c->tune_main_ms > 0.f && top_ms * 1000.0 < static_cast<double>(kRefineOverMainPermille) * c->tune_main_ms)
        return RTX_OK;
    std::vector<size_t> cand;
    for (size_t p = 0; p < np; ++p)
        if (c->h_parts[p].x >= 0 && m[p] * 1000 >= top * c->refine_top && c->h_parts[p].w < 31) cand.push_back(p);
    std::sort(cand.begin(), cand.end(), [&](size_t x, size_t y) { return m[x] > m[y]; });
    if (cand.size() > c->refine_splits) cand.resize(c->refine_splits);
    std::vector<char> cut(np, 0);
    size_t n_new = np;
    for (size_t p : cand) {
        // the part's node record (copy 0 of the node array): children only under an inner node
        float4 rec[2];
        HIP_TRY(c, hipMemcpy(rec, c->dev.nodes + 2ull * static_cast<uint32_t>(c->h_parts[p].y), sizeof rec,
                             hipMemcpyDeviceToHost));
        uint32_t link, ntri;
        std::memcpy(&link, &rec[1].z, 4);
        std::memcpy(&ntri, &rec[1].w, 4);
        if (ntri != 0 || n_new + 1 > static_cast<size_t>(kMaxParts)) continue;
        cut[p] = 1;
        ++n_new;
        // (device layout: an inner node's link is its child pair's byte offset, 32 B a slot)
        c->h_parts[p].y = static_cast<int>(link / 32u);   // the left child; the right one is inserted below
    }
    if (n_new == np) return RTX_OK;
    std::vector<int4> fr;
    fr.reserve(n_new);
    for (size_t p = 0; p < np; ++p) {
        const int4 e = c->h_parts[p];
        if (!cut[p]) {
            fr.push_back(e);
            continue;
        }
        fr.push_back(make_int4(e.x, e.y, e.z, e.w + 1));
        fr.push_back(make_int4(e.x, e.y + 1, e.z | (1 << e.w), e.w + 1));
    }
    c->h_parts.swap(fr);
    if (const int rc = join_split(c); rc != RTX_OK) return rc;   // (the chain may still read the parts)
    HIP_TRY(c, hipMemcpyAsync(c->parts_dev, c->h_parts.data(), c->h_parts.size() * sizeof(int4), hipMemcpyHostToDevice,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));   // (the host copy is replaced by the next round)
    c->dev.n_parts = static_cast<uint32_t>(c->h_parts.size());
    if (c->tune_on) {   // a shorter chain: the split factor is balanced again from where it is
        c->tune_done = false;
        c->tune_steps = 0;
        c->tune_dir = 0;
        c->tune_step = 1.15f;
        c->tune_best_span = 0.f;
        c->tune_best_permille = 0;
        c->win_state = 0;
        c->win_frames = 0;
        c->win_interval_ms = 0.f;
    }
    if (c->refine_round < c->refine_rounds) {
        c->refine_state = 0;
        c->refine_wait = 8;   // frames of the new frontier before it is measured
    }
    return RTX_OK;
}

// Whether a frame in flight (k frames of this device's contexts at once) renders one piece
// (kInflightCritPermille): its heaviest tile is short next to the split frame's serialized span, or
// the split frames in flight were measured not to overlap (their interval on this context's stream
// ~ k x the serialized span: the chain's work fills the GPU, so the frames only queue).  Times the
// interval over kInflightWindow split frames in flight first (rtx_ctx::win_*).
bool inflight_onepiece(rtx_ctx* c, uint32_t k) {
    c->win_rec = -1;
    if (c->inflight_crit == 0) return false;
    const float r = inflight_ratio(c);
    if (r > 0.f && r * 1000.f < static_cast<float>(c->inflight_crit)) return true;
    if (c->win_state == 4)   // measured: overlap = k x span / interval
        return c->tune_best_span > 0.f && c->win_interval_ms > 0.f &&
               static_cast<float>(k) * c->tune_best_span < kInflightOverlapMin * c->win_interval_ms;
    if (c->win_state == 0 && ++c->win_frames >= kInflightWindowSkip) {
        c->win_state = 2;
        c->win_frames = 0;
        c->win_rec = 0;
    } else if (c->win_state == 2 && ++c->win_frames == kInflightWindow) {
        c->win_state = 3;
        c->win_rec = 1;
    } else if (c->win_state == 3) {
        const hipError_t q = hipEventQuery(c->ev_win[1]);
        (void)hipGetLastError();   // (not-ready is no error for the caller's checks)
        if (q == hipSuccess) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, c->ev_win[0], c->ev_win[1]) == hipSuccess && ms > 0.f)
                c->win_interval_ms = ms / static_cast<float>(kInflightWindow);
            (void)hipGetLastError();
            c->win_state = 4;
        }
    }
    return false;
}
float inflight_ratio(const rtx_ctx* c) {
    if (c->max_cost_serial == 0 || c->tune_best_span <= 0.f) return 0.f;
    const float tile_ms = static_cast<float>(c->max_cost_serial) * static_cast<float>(kSplitMinUs) /
                          static_cast<float>(kSplitMinCost) * 1e-3f;
    return tile_ms / c->tune_best_span;
}

}  // namespace rtxh
