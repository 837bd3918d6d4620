// One-call codec step for a world size of 1 (host-side orchestration only; no kernels here).
//
// At world size 1 both all-reduces of the reference hook are identities
// (group_topk_hook_no_reshape.py:264, :280), so a whole call is encode -> select -> pack ->
// decode on one stream.  arctopk_step enqueues that sequence in one C call on the buffers a
// plan was bound to (arctopk_plan_bind): the hook pays one foreign-function round trip per
// call instead of one per phase.  World sizes > 1 keep the phase entry points, with the
// collectives between them.
#include "common.h"

extern "C" int arctopk_plan_bind(arctopk_plan* p, void* sketch, int32_t* rowlist, int32_t* slotmap,
                                 void* packed, void* V) {
    if (!p || !sketch || !rowlist || !slotmap || !packed) return ARCTOPK_EINVAL;
    if (p->info.v_len > 0 && !V) return ARCTOPK_EINVAL;
    p->b_sketch = sketch;
    p->b_rowlist = rowlist;
    p->b_slotmap = slotmap;
    p->b_packed = packed;
    p->b_V = V;
    return 0;
}

extern "C" int arctopk_step(const arctopk_plan* p, void* bucket, void* err, void* gerr, int32_t ef,
                            int32_t err_in, int32_t draw, uint64_t seed, const arctopk_plan* next,
                            uint64_t next_seed, void* stream) {
    if (!p || !bucket || !p->b_sketch) return ARCTOPK_EINVAL;  // unbound plan
    if (next && !next->b_sketch) return ARCTOPK_EINVAL;
    int e = 0;
    if (draw && p->info.v_len > 0) e = arctopk_draw_projections(p, seed, p->b_V, stream);
    if (!e) e = arctopk_encode(p, bucket, err, ef, err_in, p->b_V, p->b_sketch, stream);
    if (!e)
        e = arctopk_select_draw(p, p->b_sketch, 1, p->b_rowlist, p->b_slotmap, next, next_seed,
                                next ? next->b_V : nullptr, stream);
    if (!e) e = arctopk_pack(p, bucket, err, ef, p->b_rowlist, p->b_slotmap, p->b_packed, stream);
    if (!e) e = arctopk_decode(p, p->b_packed, p->b_slotmap, 1, ef, gerr, bucket, stream);
    return e;
}
