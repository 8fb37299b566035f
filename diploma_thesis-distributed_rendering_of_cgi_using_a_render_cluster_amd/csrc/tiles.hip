// k_tiles (wavefront.hip), compiled in a translation unit of its own: the
// Makefile builds this one without SLP vectorisation. Paired fp32 ops
// (v_pk_mul/add_f32) need their operands in aligned register pairs, and in the
// tile kernel's 128-VGPR budget the moves that build those pairs cost more
// VALU issue than the pairing saves: 04vs frame 5 2.33 -> 2.18 ms. The split
// path kernels keep SLP (k_trace_primary +46 % without it, 02 frame 60).
// Same arithmetic op for op either way (-ffp-contract=off in both TUs).
#define RR_TILES_TU 1
#include "wavefront.hip"
