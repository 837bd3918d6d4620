// Diagnostic: phase timestamps of the fused select on the headline plan (16 x [2048,2048]).
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -DARCTOPK_SEL_STAMPS -Iinclude -Iallreducetopk_amd/csrc scripts/seltest.hip -o scripts/seltest
#include "../allreducetopk_amd/csrc/plan.hip"
#include "../allreducetopk_amd/csrc/arctopk_kernels.hip"
#include "../allreducetopk_amd/csrc/mselect.hip"
#include "../allreducetopk_amd/csrc/vdraw.hip"
#include <cstdio>
#include <vector>
#include <random>
int main() {
    std::vector<int64_t> dims;
    std::vector<int32_t> nd;
    for (int i = 0; i < 16; ++i) { dims.push_back(2048); dims.push_back(2048); nd.push_back(2); }
    arctopk_plan* p;
    if (arctopk_plan_create(dims.data(), nd.data(), 16, 4, 0.2, 0, 0, &p)) return 1;
    arctopk_plan_info info;
    arctopk_plan_query(p, &info);
    std::vector<float> sk(info.sketch_len);
    std::mt19937 rng(1);
    std::normal_distribution<float> nd01;
    for (auto& x : sk) x = nd01(rng) * 30.f;
    float* dsk; int32_t *rl, *sm;
    (void)hipMalloc(&dsk, sk.size() * 4);
    (void)hipMalloc(&rl, info.sel_rows * 4);
    (void)hipMalloc(&sm, info.rows_total * 4);
    (void)hipMemcpy(dsk, sk.data(), sk.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        arctopk_select(p, dsk, 1, rl, sm, nullptr);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long st[64];
        (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_sel_stamps), sizeof(st));
        printf("rep %d: %.2f us | load+energy %llu, or/and %llu, hist %llu, gather %llu, rank %llu, radix-total %llu, scan %llu, write %llu (s_memtime ticks)\n", rep, ms * 1e3,
               st[8] - st[0], st[1] - st[8], st[5] - st[1], st[6] - st[5], st[7] - st[6], st[2] - st[1], st[3] - st[2], st[4] - st[3]);
    }
    return 0;
}
