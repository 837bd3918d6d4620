// Select-only timing harness (diagnostic; not product code): builds the plan of a shape set,
// encodes a Gaussian bucket with Gaussian projections through the library (realistic sketch
// energies), then times arctopk_select alone.  Variants are compiled with -D switches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iallreducetopk_amd/csrc \
//     scripts/selbench.hip allreducetopk_amd/csrc/{plan,arctopk_kernels,mselect}.hip -o scripts/selbench
//   ./scripts/selbench resnet50|resnet18b0|resnet18b1|llama|roberta|headline [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "arctopk.h"
#ifdef ARCTOPK_STAMPS
extern "C" int arctopk_diag_stamps_k(int which, unsigned long long* host);
extern "C" int arctopk_diag_stamps_m(int which, unsigned long long* host);
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

static void add(std::vector<int64_t>& d, std::vector<int32_t>& nd, std::initializer_list<int64_t> s) {
    for (int64_t x : s) d.push_back(x);
    nd.push_back((int32_t)s.size());
}

int main(int argc, char** argv) {
    const std::string which = argc > 1 ? argv[1] : "resnet50";
    const int reps = argc > 2 ? atoi(argv[2]) : 30;
    std::vector<int64_t> dims;
    std::vector<int32_t> nd;
    if (which == "resnet50") {
        for (int g = 0; g < 3; ++g) {
            add(dims, nd, {2048}); add(dims, nd, {2048}); add(dims, nd, {2048, 512, 1, 1});
            add(dims, nd, {512}); add(dims, nd, {512}); add(dims, nd, {512, 512, 3, 3});
            add(dims, nd, {512}); add(dims, nd, {512}); add(dims, nd, {512, 2048, 1, 1});
        }
        add(dims, nd, {2048, 1024, 1, 1});
    } else if (which == "resnet18b0") {  // first DDP bucket: fc + last block's bn/conv
        add(dims, nd, {10}); add(dims, nd, {10, 512}); add(dims, nd, {512}); add(dims, nd, {512});
        add(dims, nd, {512, 512, 3, 3});
    } else if (which == "resnet18b1") {
        add(dims, nd, {512}); add(dims, nd, {512}); add(dims, nd, {512, 512, 3, 3});
        add(dims, nd, {512}); add(dims, nd, {512}); add(dims, nd, {512, 256, 1, 1});
        add(dims, nd, {512}); add(dims, nd, {512}); add(dims, nd, {512, 512, 3, 3});
        add(dims, nd, {512}); add(dims, nd, {512}); add(dims, nd, {512, 256, 3, 3});
        add(dims, nd, {256}); add(dims, nd, {256}); add(dims, nd, {256, 256, 3, 3});
    } else if (which == "llama") {
        add(dims, nd, {32000, 2048});
    } else if (which == "roberta") {
        add(dims, nd, {50265, 768});
    } else {
        for (int i = 0; i < 16; ++i) add(dims, nd, {2048, 2048});
    }
    arctopk_plan* p = nullptr;
    int st = arctopk_plan_create(dims.data(), nd.data(), (int)nd.size(), 4, 0.2, ARCTOPK_F32, 0, &p);
    if (st) { printf("plan_create %d\n", st); return 1; }
    arctopk_plan_info info;
    arctopk_plan_query(p, &info);
    std::mt19937 rng(7);
    std::normal_distribution<float> n01;
    std::vector<float> hG(info.numel), hV(info.v_len);
    for (auto& x : hG) x = n01(rng);
    if (const char* zr = getenv("ZERO_ROWS")) {  // ZERO_ROWS=m: 9 of every 10 rows of m values all zero
        const int64_t m = atoll(zr);
        for (int64_t i = 0; i < (int64_t)hG.size(); ++i)
            if ((i / m) % 10 != 0) hG[i] = 0.f;
    }
    for (auto& x : hV) x = n01(rng);
    float *G, *V, *sk;
    int32_t *rl, *sm;
    CK(hipMalloc(&G, info.numel * 4));
    CK(hipMalloc(&V, std::max<int64_t>(1, info.v_len) * 4));
    CK(hipMalloc(&sk, info.sketch_len * 4));
    CK(hipMalloc(&rl, info.sel_rows * 4));
    CK(hipMalloc(&sm, info.rows_total * 4));
    CK(hipMemcpy(G, hG.data(), info.numel * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(V, hV.data(), info.v_len * 4, hipMemcpyHostToDevice));
    st = arctopk_encode(p, G, nullptr, ARCTOPK_EF_NONE, 1, V, sk, nullptr);
    if (st) { printf("encode %d\n", st); return 1; }
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    const bool evict = getenv("EVICT") != nullptr;  // stream 512 MiB between selects (cold L2 / I-cache)
    void* big = nullptr;
    if (evict) CK(hipMalloc(&big, (size_t)512 << 20));
    for (int r = 0; r < reps; ++r) {
        if (evict) CK(hipMemsetAsync(big, r & 0xFF, (size_t)512 << 20, nullptr));
        CK(hipEventRecord(e0, nullptr));
        st = arctopk_select(p, sk, 1, rl, sm, nullptr);
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        if (st) { printf("select %d\n", st); return 1; }
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    // check: k selected rows per segment, slot map consistent
    std::vector<int32_t> hsm(info.rows_total);
    CK(hipMemcpy(hsm.data(), sm, info.rows_total * 4, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int i = 0; i < info.nseg; ++i) {
        arctopk_segment s;
        arctopk_plan_segment(p, i, &s);
        int64_t c = 0;
        for (int64_t r = 0; r < s.n; ++r) c += hsm[s.row_off + r] >= 0;
        bad += c != s.k_rows;
    }
    printf("%-11s rows %9lld segs %3d select median %8.2f us  min %8.2f  %s\n", which.c_str(),
           (long long)info.rows_total, info.nseg, ts[ts.size() / 2], ts[0], bad ? "BAD COUNTS" : "ok");
#ifdef ARCTOPK_STAMPS
    {   // per-block timeline of the last select (ticks of 10 ns, relative to the key pass start)
        const size_t NS = 4096 * 8;
        std::vector<unsigned long long> st[4];
        for (auto& v : st) v.assign(NS, 0ull);
        for (int k = 0; k < 2; ++k) {
            CK((hipError_t)arctopk_diag_stamps_k(k, st[k == 0 ? 0 : 2].data()));
            CK((hipError_t)arctopk_diag_stamps_m(k, st[k == 0 ? 1 : 3].data()));
        }
        const char* names[4] = {"keys", "compact", "refine", "write"};
        unsigned long long t0 = ~0ull;
        for (size_t b = 0; b < 4096 && st[0][b * 8]; ++b) t0 = std::min(t0, st[0][b * 8]);
        for (int k = 0; k < 4; ++k) {
            std::vector<double> dur, s01, s12, s23;
            unsigned long long smin = ~0ull, smax = 0, emax = 0;
            int nb = 0;
            for (size_t b = 0; b < 4096; ++b) {
                const unsigned long long* e = &st[k][b * 8];
                if (!e[0] || e[0] < t0) break;
                ++nb;
                const int last = (k == 0) ? 3 : 1;
                smin = std::min(smin, e[0]);
                smax = std::max(smax, e[0]);
                emax = std::max(emax, e[last]);
                dur.push_back((double)(e[last] - e[0]) * 0.01);
                if (k == 0) {
                    s01.push_back((e[1] - e[0]) * 0.01);
                    s12.push_back((e[2] - e[1]) * 0.01);
                    s23.push_back((e[3] - e[2]) * 0.01);
                }
            }
            auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
            auto mx = [](const std::vector<double>& v) { double m = 0; for (double x : v) m = std::max(m, x); return m; };
            printf("  %-8s blocks %5d  start %7.2f .. %7.2f us  end %7.2f us  block med %6.2f max %6.2f",
                   names[k], nb, (smin - t0) * 0.01, (smax - t0) * 0.01, (emax - t0) * 0.01, med(dur), mx(dur));
            if (k == 2) {  // refine items (blocks 0 .. nitems-1 write slots 2-4)
                for (size_t b = 0; b < 64; ++b) {
                    const unsigned long long* e = &st[2][b * 8];
                    if (!e[2] || e[2] < e[0]) break;
                    if (e[5] > e[0] && e[5] < e[1]) printf("\n    item %2zu: first pass %.2f, second pass %.2f", b, (e[5] - e[0]) * 0.01, (e[1] - e[5]) * 0.01);
                    printf("\n    item %2zu: stage %.2f rounds %.2f count %.2f offsets %.2f (start %.2f)", b,
                           (e[2] - e[0]) * 0.01, (e[3] - e[2]) * 0.01, (e[4] - e[3]) * 0.01, (e[1] - e[4]) * 0.01,
                           (e[0] - t0) * 0.01);
                }
            }
            if (k == 0) {  // per item: blocks, median / max load+hist, max end
                std::map<int, std::vector<double>> lh, en;
                for (size_t b = 0; b < (size_t)nb; ++b) {
                    const unsigned long long* e = &st[0][b * 8];
                    lh[(int)e[4]].push_back((e[1] - e[0]) * 0.01);
                    en[(int)e[4]].push_back((e[3] - t0) * 0.01);
                }
                for (auto& kv : lh)
                    printf("\n    item %2d: blocks %4zu load+hist med %6.2f max %6.2f  end max %6.2f", kv.first,
                           kv.second.size(), med(kv.second), mx(kv.second), mx(en[kv.first]));
            }
            if (k == 0) printf("  [load+hist med %.2f max %.2f | merge med %.2f max %.2f | arrive/digit max %.2f]",
                               med(s01), mx(s01), med(s12), mx(s12), mx(s23));
            printf("\n");
        }
    }
#endif
    return 0;
}
