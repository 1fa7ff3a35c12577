// host_build_timer.cpp — times the host Update of one animated mesh (transform, then the
// fast BVH build) without HIP, so the builder can be A/B'd on the GPU box's CPU:
//   g++ -std=c++17 -O3 -ffp-contract=off -fno-fast-math -pthread -Igp1_raytracer_2223_amd/csrc/host
//       -Iinclude tools/host_build_timer.cpp gp1_raytracer_2223_amd/csrc/host/scene.cpp -o tools/hb_tmp/timer
//   RTX_HOST_THREADS=8 RTX_HOST_PAR_TRIS=128 tools/hb_tmp/timer gp1_raytracer_2223_amd/assets [scene]
// (results: profiles/r02/host_update_fork_thresholds.txt)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "scene.h"

using namespace rtx;

int main(int argc, char** argv) {
    if (argc < 2) {
        std::printf("usage: %s <asset dir> [scene]\n", argv[0]);
        return 2;
    }
    auto s = MakeScene(argc > 2 ? argv[2] : "W4_Optional", argv[1]);
    if (!s || !s->Initialize() || s->Spinning().empty()) {
        std::printf("init failed\n");
        return 1;
    }
    TriangleMesh* m = s->Spinning()[0];
    using clk = std::chrono::steady_clock;
    const int n = 600, warm = 20;
    double tt = 0;
    std::vector<double> bs;
    for (int k = 0; k < n + warm; ++k) {
        m->RotateY(0.01f * k);
        const auto t0 = clk::now();
        // TriangleMesh::UpdateTransforms without its BuildBVH, so the two phases time apart
        const Mat4 f = m->scaleTransform * m->rotationTransform * m->translationTransform;
        m->transformedPositions.clear();
        for (const auto& p : m->positions) m->transformedPositions.push_back(f.TransformPoint(p));
        m->transformedNormals.clear();
        for (const auto& q : m->normals) m->transformedNormals.push_back(f.TransformVector(q).Normalized());
        const auto t1 = clk::now();
        m->BuildBVH();
        const auto t2 = clk::now();
        if (k >= warm) {
            tt += std::chrono::duration<double>(t1 - t0).count();
            bs.push_back(std::chrono::duration<double>(t2 - t1).count());
        }
    }
    double tb = 0;
    for (double b : bs) tb += b;
    std::sort(bs.begin(), bs.end());
    std::printf("transform %.1f us, build mean %.1f us, p10 %.1f, median %.1f\n", tt / n * 1e6, tb / n * 1e6,
                bs[n / 10] * 1e6, bs[n / 2] * 1e6);
}
