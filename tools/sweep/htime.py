#!/usr/bin/env python3
"""Generate the timestamped (diagnostic) build source of the hierarchy kernels from the PRODUCT
source: flame_amd/csrc/fedagg.hip with per-workgroup s_memrealtime stamps (100 MHz) inserted at
fixed anchors.  Every anchor must match exactly once, so a change of the product source that
moves one fails here instead of silently stamping the wrong place.  Nothing else changes: the
stamped kernels compute the same bits (tools/hier_attrib.py checks), they only also store the
stamps into the buffer flame_sweep_htime() names (vector stores from one lane).

Slots per workgroup (the layout tools/hier_attrib.py reads; M middles, NB = ceil(M / 16) groups):
  hier_fedbuff_body (LDS store groups), wave 0 lane 0:
    0 start, 1 end, 2 HW_ID | XCC_ID << 32, 3 + 2m the end of middle m's reduction,
    4 + 2m the end of its epilogue, 3 + 2M + g the end of store burst g
(Round 5's wave-specialised variant, hier_ws_body, had stamps of its own; it left the product
source with its measurement)

    python tools/sweep/htime.py OUT.hip
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "flame_amd", "csrc", "fedagg.hip")

HELPERS = r'''
// ---- DIAGNOSTIC BUILD (tools/sweep/htime.py): per-workgroup timestamps
__device__ uint64_t* g_htime = nullptr;
__device__ int g_htime_slots = 0;
__device__ __forceinline__ void htime_at(bool who, int slot, uint64_t v) {
    if (who && g_htime && slot < g_htime_slots)
        g_htime[static_cast<int64_t>(blockIdx.x) * g_htime_slots + slot] = v;
}
#define FLAME_HT(who, slot) htime_at((who), (slot), __builtin_amdgcn_s_memrealtime())
#define FLAME_HW(who)                                                                                \
    htime_at((who), 2, static_cast<uint64_t>(__builtin_amdgcn_s_getreg((31 << 11) | 4)) |           \
                           (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((15 << 11) | 20)) << 32))
'''

EXPORT = r'''
// Diagnostic builds only: where the hierarchy kernels write their timestamps (NULL = nowhere).
extern "C" int flame_sweep_htime(void* buf, int32_t slots) {
    uint64_t* p = static_cast<uint64_t*>(buf);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_htime), &p, sizeof(p));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_htime_slots), &slots, sizeof(slots));
    return e == hipSuccess ? 0 : 2;
}
'''

W0 = "threadIdx.x == 0"

# (anchor, replacement) -- the anchor text is kept, the stamp goes before or after it
EDITS = [
    # helpers after the rounding helpers' section header
    ("// ---------------------------------------------------------------- rounding helpers\n",
     HELPERS + "// ---------------------------------------------------------------- rounding helpers\n"),
    # hier_fedbuff_body: start + hw id at the vector path's entry
    ("    const T* tin = reinterpret_cast<const T*>(sg.top_agg_in) + e0;\n    if (vec) {\n        if (have_top) {\n",
     "    const T* tin = reinterpret_cast<const T*>(sg.top_agg_in) + e0;\n    if (vec) {\n"
     f"        FLAME_HT({W0}, 0);\n        FLAME_HW({W0});\n        if (have_top) {{\n"),
    ("            reduce_clients<DT, CU, true>(acc, !SYNC, crow + static_cast<int64_t>(m) * n_clients, n_clients,\n"
     "                                         mid_rates + static_cast<int64_t>(m) * n_clients, nullptr, e0, sg.numel,\n"
     "                                         coff);\n",
     "            reduce_clients<DT, CU, true>(acc, !SYNC, crow + static_cast<int64_t>(m) * n_clients, n_clients,\n"
     "                                         mid_rates + static_cast<int64_t>(m) * n_clients, nullptr, e0, sg.numel,\n"
     f"                                         coff);\n            FLAME_HT({W0}, 3 + 2 * m);\n"),
    ("                if (dp) st_v(dp + v * VS, pack<T, EPT>(d));\n            }\n            have_top = true;\n            }\n",
     "                if (dp) st_v(dp + v * VS, pack<T, EPT>(d));\n            }\n            have_top = true;\n"
     f"            FLAME_HT({W0}, 4 + 2 * m);\n            }}\n"),
    ("                        st_v(wp + v * VS, pv);\n                    }\n                }\n            }\n        }\n",
     "                        st_v(wp + v * VS, pv);\n                    }\n                }\n            }\n"
     f"            FLAME_HT({W0}, 3 + 2 * n_mids + m0 / HB);\n        }}\n"),
    ("                st_v(gp, pack<T, EPT>(gw));\n            }\n        }\n        return;\n    }\n"
     "    hier_tail<DT, SYNC>(",
     "                st_v(gp, pack<T, EPT>(gw));\n            }\n        }\n"
     f"        FLAME_HT({W0}, 1);\n        return;\n    }}\n    hier_tail<DT, SYNC>("),
]


def generate(out):
    s = open(SRC).read()
    for i, (anchor, repl) in enumerate(EDITS):
        n = s.count(anchor)
        if n != 1:
            raise SystemExit(f"tools/sweep/htime.py: anchor {i} matches {n} times in {SRC} (expected 1): "
                             f"{anchor[:90]!r}...")
        s = s.replace(anchor, repl)
    s = s.replace('#include "../../include/flame_amd.h"', f'#include "{os.path.join(ROOT, "include", "flame_amd.h")}"')
    s = s.replace('#include "fastmath.h"', f'#include "{os.path.join(ROOT, "flame_amd", "csrc", "fastmath.h")}"')
    s += EXPORT
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        f.write(s)
    return out


if __name__ == "__main__":
    generate(sys.argv[1])
