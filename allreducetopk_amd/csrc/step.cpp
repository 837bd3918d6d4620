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

// arctopk_step (the cached-graph step) lives with the kernels it launches (arctopk_kernels.hip).
