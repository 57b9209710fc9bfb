// tuning.hpp -- the library's measurement knobs (CLAY_* environment variables), read ONCE when
// libclay_amd.so is loaded (a namespace-scope initialiser in code.cpp), never on a call path.
// The reference's ClayCode is immutable and Send + Sync (/root/reference/src/lib.rs:58): no
// encode / decode / repair call may depend on process-wide mutable state such as the
// environment (setenv racing getenv is undefined behaviour).  Behaviour that tests must switch
// at run time goes through the ABI (clay_set_exec_mode, clay_set_encode_path) instead.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace clay {

struct Tuning {
    // planner (plan.cpp); < 0: the built-in default
    int plan_inline = 1;         // CLAY_PLAN_INLINE=0 disables input inlining
    int plan_dup = -1;           // CLAY_PLAN_DUP
    int plan_fold_cost = -1;     // CLAY_PLAN_FOLD_COST
    int plan_defer_out = -1;     // CLAY_PLAN_DEFER_OUT
    int plan_merge_slack = -1;   // CLAY_PLAN_MERGE_SLACK
    bool plan_debug = false;     // CLAY_PLAN_DEBUG (stderr dump of plans)
    // grouped / tile executors (engine.hip)
    int texec_waves = 0;         // CLAY_TEXEC_WAVES (4 / 8 / 16; 0 = by plan)
    size_t texec_lds = 80 * 1024;  // CLAY_TEXEC_LDS_KB
    bool texec_big = false;      // CLAY_TEXEC_BIG
    bool gexec_pipe = true;      // CLAY_GEXEC_PIPE=0 disables the software pipeline
    uint32_t gexec_order = 2;    // CLAY_GEXEC_ORDER
    int gexec_tpw = 0;           // CLAY_GEXEC_TPW (1..64; 0 = per level)
    uint64_t gexec_small = 2048; // CLAY_GEXEC_SMALL
    uint64_t gexec_big = 32768;  // CLAY_GEXEC_BIG
    // host pipeline
    size_t host_piece = size_t(256) << 20;  // CLAY_HOST_PIECE_MB
    int host_streams = 2;                   // CLAY_HOST_STREAMS
    // probe library only (libclay_amd_probe.so): decode kernel parts to skip
    int decode_probe = 0;        // CLAY_DECODE_PROBE
    // streaming decodes: LDS node buffers of the ring (6..10; the split syn kernel and the local
    // kernel use one less, the last holds the tables)
    uint32_t decode_ring = 10;   // CLAY_DECODE_RING
    // local decode: the 64-byte-tile kernel also for one erasure in section G (A/B measurements)
    bool local_w64 = false;      // CLAY_LOCAL_W64
};

// The knobs as read at load time.
const Tuning &tuning();

}  // namespace clay
