// pbr_config.h — the build's tuning switches.
//
// Every kernel parameter below has ONE measured default (DESIGN.md §4/§7 give the A/B numbers).
// Release builds take the defaults only: overriding a switch from the command line is an error
// unless the build opts into development knobs with -DPBR_DEV_KNOBS=1 (what the A/B scripts in
// tools/ do), so the shipped libpbr_hip.so has a single schedule and reads no environment.  The
// run-time choices that remain — chunk size, lanes, megakernel vs wavefront, level-0 fusion — are
// explicit arguments of pbr_hip_set_schedule (include/pbr_hip.h), each covered by the GPU tests.
#pragma once

#if !defined(PBR_DEV_KNOBS) || !PBR_DEV_KNOBS
#if defined(PBR_TRAV_DIAG) || defined(PBR_HELPER) || defined(PBR_SHORT_STACK_DEPTH) || defined(PBR_TRAV_OCC) ||   \
    defined(PBR_REFILL_SHORT) || defined(PBR_SCALAR_LOADS) || defined(PBR_QUAD_TRAVERSAL) || defined(PBR_PACKET) || \
    defined(PBR_PACKET_EXTEND) || defined(PBR_XCD_RUN) || defined(PBR_XCD_TRAV_RUN) || defined(PBR_REFILL) ||       \
    defined(PBR_REFILL_OCC) || defined(PBR_REFILL_OCC_ANY) || defined(PBR_REFILL_OCC_TR) ||                          \
    defined(PBR_CAMERA_SHORT) || defined(PBR_WF_SHADE_OCC) || defined(PBR_WF_SHADE_OCC_MM) ||                        \
    defined(PBR_WF_FUSED_OCC) || defined(PBR_WFP_OCC) || defined(PBR_WFV_OCC) || defined(PBR_LANES_DEFAULT) ||       \
    defined(PBR_INLINE_TRANS) || defined(PBR_DIAG_SHADE) || defined(PBR_STACK_DIAG) || defined(PBR_ANY_SHORT) || defined(PBR_WF_BLOCKS) || defined(PBR_CLASSED_SHADE) || defined(PBR_WF_FUSED_MATS_LDS) || defined(PBR_WFP_OCC_MM) || defined(PBR_WFP_OCC_L) || \
    defined(PBR_NF_ROWS) || defined(PBR_SEG_WAVE) || defined(PBR_SLAB_BRANCHLESS) || defined(PBR_WF_WHITTED_MAXLOG2) || defined(PBR_OWN_LANES)
#error "tuning switches are development builds only: add -DPBR_DEV_KNOBS=1"
#endif
#endif
// PBR_DIAG_SHADE (diagnostic builds only, results NOT the reference's): bits that stub parts of the
// Path shade to price them (tools/r5_shade_probe.py).
#ifndef PBR_DIAG_SHADE
#define PBR_DIAG_SHADE 0
#endif
// PBR_STACK_DIAG (diagnostic builds): the lane-refill traversals count the rays whose stack went
// deeper than 6 / 10 / 16 / 24 entries into profile fields 2-5 of their family.
#ifndef PBR_STACK_DIAG
#define PBR_STACK_DIAG 0
#endif
// Path: one shade launch per material lobe set when the scene's materials have several (k_wfp_shade
// CLASSED)
#ifndef PBR_CLASSED_SHADE
#define PBR_CLASSED_SHADE 1
#endif
