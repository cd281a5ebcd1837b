/* yk_test_hooks.h — test-only entry points of libyk.so. NOT part of the
 * product ABI (include/yk_api.h): a plugin never includes this header.
 * Every hook here refuses to run (YK_ERR_UNSUPPORTED) unless the process
 * environment has YK_DEBUG_HOOKS=1, so an integrator cannot damage a device
 * by accident. */
#ifndef YK_TEST_HOOKS_H
#define YK_TEST_HOOKS_H
#include "yk_api.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Test hook for the traversal watchdog: overwrites node `index` of the
 * device's resident kd-tree with the export-encoding words (w0, w1), as a
 * memory fault would, past the structural check yk_device_upload applies.
 * Child and leaf ranges must still lie inside the tree (YK_ERR_ARG
 * otherwise), so the damage is structural (a cycle, a shared subtree, a
 * deeper descent); ray queries and renders on the damaged tree must then
 * return YK_ERR_INTERNAL within seconds, never hang or fault. A fresh
 * yk_device_upload restores the device. YK_ERR_UNSUPPORTED unless
 * YK_DEBUG_HOOKS=1. */
int yk_device_debug_set_node(yk_device* d, int64_t index, uint32_t w0, uint32_t w1);

/* QMC / fast-math probe: runs one of libyk's restatements of the reference's
 * header-only functions over n inputs (host pointers), so tests can compare
 * them with the reference's own functions compiled in the build container
 * (tests/golden/ref_qmc.npz). Device functions (yk_math.h and the film's
 * rounding) run in a kernel on `d`; the HOST_* ones are the host-side copies
 * libyk uses for the film's filter tables and need no device.
 *   RI_VDC / RI_S / RI_LP  in: u32 index, in2: u32 scramble -> f32   (mcqmc.h:100-122)
 *   FNV                    in: u32 -> u32                            (mcqmc.h:155)
 *   FSIN / FCOS, HOST_FSIN in: f32 -> f32                   (mathOptimizations.h:249-280)
 *   HALTON2/3/5            in: u32 start -> 8 f32 (setStart, 8x getNext; mcqmc.h:29-94)
 *   ROUND2INT / FLOOR2INT  in: f64 -> i32                   (math_utils.h:60-86)
 *   HOST_FEXP2             in: f32 -> f32                   (mathOptimizations.h:100)
 * YK_ERR_UNSUPPORTED unless YK_DEBUG_HOOKS=1. */
enum {
  YK_PROBE_RI_VDC = 0, YK_PROBE_RI_S = 1, YK_PROBE_RI_LP = 2, YK_PROBE_FNV = 3, YK_PROBE_FSIN = 4,
  YK_PROBE_FCOS = 5, YK_PROBE_HALTON2 = 6, YK_PROBE_HALTON3 = 7, YK_PROBE_HALTON5 = 8,
  YK_PROBE_ROUND2INT = 9, YK_PROBE_FLOOR2INT = 10, YK_PROBE_HOST_FEXP2 = 11, YK_PROBE_HOST_FSIN = 12
};
int yk_debug_qmc_probe(yk_device* d, int32_t fn, const void* in, const uint32_t* in2, int64_t n, void* out);

/* Which traversal kernels the resident scene takes: *bytes = the size of the
 * LDS copy of its traversal data when ray queries and renders run the
 * small-scene kernels (node packets and triangle records in LDS), 0 when
 * they read them from HBM. YK_ERR_UNSUPPORTED unless YK_DEBUG_HOOKS=1. */
int yk_debug_small_scene(yk_device* d, int64_t* bytes);

/* Which shading instantiation the resident scene takes: *diff_only = 1 when
 * the shading and final-gather kernels run the diffuse-only specialisation
 * (mat_sample<true>: every material a light or a one-component diffuse
 * shinydiffuse, and YK_DIFF != 0 at upload), 0 for the general component
 * loop. YK_ERR_UNSUPPORTED unless YK_DEBUG_HOOKS=1. */
int yk_debug_shading_kind(yk_device* d, int32_t* diff_only);

/* Which form a render of the resident scene with params p gives its shadow
 * slots: *split = 1 for 16-B direction records plus one origin per shading
 * point (any-hit kernels k_trace_shadow[_small]_split), 0 for whole 32-B
 * rays. YK_ERR_UNSUPPORTED unless YK_DEBUG_HOOKS=1. */
int yk_debug_shadow_form(yk_device* d, const yk_render_params* p, int32_t* split);

#ifdef __cplusplus
}
#endif
#endif /* YK_TEST_HOOKS_H */
