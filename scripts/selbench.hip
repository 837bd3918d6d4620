// Select-only timing harness (diagnostic; not product code): builds the plan of a shape set,
// encodes a Gaussian bucket with Gaussian projections through the library (realistic sketch
// energies), then times arctopk_select alone.  Variants are compiled with -D switches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iallreducetopk_amd/csrc \
//     scripts/selbench.hip allreducetopk_amd/csrc/{plan,arctopk_kernels,mselect}.hip -o scripts/selbench
//   ./scripts/selbench resnet50|resnet18b0|resnet18b1|llama|roberta|headline [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "arctopk.h"

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
    for (int r = 0; r < reps; ++r) {
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
    return 0;
}
