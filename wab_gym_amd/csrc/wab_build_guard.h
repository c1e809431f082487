// wab_build_guard.h — product and diagnostic builds of the same sources.
//
// The kernels carry diagnostic switches for tools/ (stamps, store-floor and ablation builds whose
// results are wrong by design).  A stray -D of one of them in the product build would break
// parity silently, so:
//   * __graft_entry__.build() compiles with -DWAB_PRODUCT_BUILD: any diagnostic macro is an error;
//   * a diagnostic build must say so with -DWAB_DIAGNOSTIC_BUILD (tools/build_variants.sh,
//     tools/phase_stamps.py do) and goes to a path outside wab_gym_amd/_lib/libwab_hip.so; its
//     library then exports wab_diagnostic_build(), which wab_gym_amd/_lib.py refuses to load
//     unless WAB_DIAGNOSTIC_OK=1 (set only by the tools that run such builds).
#pragma once

#if defined(WAB_STAMPS) || defined(WAB2_STAMPS) || defined(WAB_ROLL_FLOOR) || defined(WAB_WIDE_ROLL_FLOOR) || \
    defined(WAB2_ABLATE) || defined(WAB_ONLY_WAVE)
#if defined(WAB_PRODUCT_BUILD)
#error "a diagnostic macro (WAB_STAMPS, WAB2_STAMPS, WAB_ROLL_FLOOR, WAB_WIDE_ROLL_FLOOR, WAB2_ABLATE, WAB_ONLY_WAVE) is set in the product build"
#elif !defined(WAB_DIAGNOSTIC_BUILD)
#error "diagnostic macros need -DWAB_DIAGNOSTIC_BUILD and an output outside the product library (tools/build_variants.sh)"
#endif
#endif

#if defined(WAB_DIAGNOSTIC_BUILD) && !defined(__HIP_DEVICE_COMPILE__)
// (weak: every translation unit of a diagnostic build defines it)
extern "C" __attribute__((weak, visibility("default"))) int wab_diagnostic_build(void) { return 1; }
#endif
