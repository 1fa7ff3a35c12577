// benchmark.h — the reference's F6 benchmark (Timer::StartBenchmark / Timer::Update,
// source/Timer.cpp:44-131), shared by the headless frame loop (rtx_render) and the viewer (rtx_view).
#pragma once
#include <algorithm>
#include <cfloat>
#include <fstream>
#include <iostream>
#include <numeric>
#include <vector>

namespace rtx {

// Timer::StartBenchmark / Update FPS logic (Timer.cpp:44-131), same float arithmetic: one-second
// dFPS windows; Tick() returns true when the last of `frames` windows closed (HIGH / LOW / AVG set).
struct Benchmark {
    int frames;
    std::vector<float> dfps;
    float high = FLT_MIN, low = FLT_MAX, avg = 0.f;   // m_BenchmarkHigh = FLT_MIN as in the reference
    float fps_timer = 0.f;
    int fps_count = 0;
    explicit Benchmark(int n) : frames(n) {}
    bool Tick(float elapsed) {   // returns true when the last window closed
        fps_timer += elapsed;
        ++fps_count;
        if (fps_timer >= 1.0f) {
            const float d = fps_count / fps_timer;
            fps_count = 0;
            fps_timer = 0.f;
            return Record(d);
        }
        return false;
    }
    // one closed window's dFPS (m_Benchmarks[m_BenchmarkCurrFrame] = m_dFPS ...); true when the
    // last window closed (AVG set)
    bool Record(float d) {
        dfps.push_back(d);
        low = std::min(low, d);
        high = std::max(high, d);
        if (static_cast<int>(dfps.size()) >= frames) {
            avg = std::accumulate(dfps.begin(), dfps.end(), 0.f) / float(frames);
            return true;
        }
        return false;
    }
};

// the benchmark's end (Timer.cpp:109-124): the three lines on stdout and benchmark.txt
inline void WriteBenchmark(const Benchmark& b) {
    std::cout << "**BENCHMARK FINISHED**\n";
    std::cout << ">> HIGH = " << b.high << std::endl;
    std::cout << ">> LOW = " << b.low << std::endl;
    std::cout << ">> AVG = " << b.avg << std::endl;
    std::ofstream out("benchmark.txt");
    out << "FRAMES = " << b.dfps.size() << std::endl;
    out << "HIGH = " << b.high << std::endl;
    out << "LOW = " << b.low << std::endl;
    out << "AVG = " << b.avg << std::endl;
}

}  // namespace rtx
