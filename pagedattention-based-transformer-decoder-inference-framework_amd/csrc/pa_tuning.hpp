// The A/B switches of the attention launches (pa_decode.hip), in ONE table.
// The product library is compiled against the constant defaults below: every
// switch folds away.  The tuning build (make tune, -DLLM_TUNING=1) reads them
// from the environment per launch and may route a beam-group launch to one of
// the experiment kernels (csrc/tune/pa_decode_tune.hip); nothing else in the
// product sources depends on LLM_TUNING for attention.
#pragma once

#include "common.hpp"

namespace llm {

struct PaSplitArgs;

struct PaTuning {
  bool wg_merge = true;        // LLM_WG_MERGE=0: split + merge launches, no workgroup merge
  bool oproj_fuse = true;      // LLM_OPROJ_FUSE=0: the FP16 o_proj GEMM launch again
  bool beam4 = false;          // LLM_BEAM4=1: pa_beam4_kernel for beam groups
  bool beam_mfma = false;      // LLM_BEAM_MFMA=1: pa_beam_mfma_kernel for beam groups
  bool beam_steal = false;     // LLM_BEAM_STEAL=1: tiles assigned while the launch runs
  int beam_balance16 = 44;     // LLM_BEAM_BALANCE16: private-tile cost, 1/16ths (0: off);
                               // sweep in DESIGN.md §9 (C4 launch 84 -> 66 us)
  int beam_mfma_balance16 = 64;  // LLM_BEAM_MFMA_BALANCE16
  int beam_nsplit = 0;         // LLM_BEAM_NSPLIT: forced split count of beam-group launches
  int wgm_splits = 0;          // LLM_WGM_SPLITS: forced split count of workgroup-merge launches
  int beam4_splits = 0;        // LLM_BEAM4_SPLITS: forced split count of pa_beam4_kernel
  bool beam_smaj = true;       // LLM_BEAM_SMAJ=0: beam workgroups in (group, head)-major order
};

// The steal form's exchange splits a shared page's 2 NI pieces of 1 KiB over
// the 4 waves: NI = TS D / 512 even (fp16 pages of 2, 4 or 8 KiB).
constexpr bool steal_shape_ok(int D, int TS) {
  return D >= 8 && D <= 512 && (TS * D) % 1024 == 0 && TS * D * 2 <= 8192;
}

#if LLM_TUNING
PaTuning pa_tuning();
// An experiment form of a beam-group split launch (pa_beam4_kernel, the steal
// form, the MFMA beam kernel, the loads-only / stamped / LDS-DMA ring variants
// of the shipped form) when its switch is on: launches it, *e = its status,
// returns true.  false: the shipped form runs.
bool tune_launch_form(const PaSplitArgs& a, int D, int TS, dim3 grid, hipStream_t st,
                      hipError_t* e);
long long tune_beam4_resident_for(int D, int TS);
// the MFMA beam kernel's occupancy when LLM_BEAM_MFMA=1 (true; *e its status)
bool tune_beam_occupancy(int D, int TS, int* blocks, hipError_t* e);
// counters of standalone steal launches (no decoder-owned ones; launches must
// not overlap), nullptr unless LLM_BEAM_STEAL=1
unsigned* tune_steal_counters(size_t n);
#else
constexpr PaTuning pa_tuning() { return PaTuning{}; }
inline bool tune_launch_form(const PaSplitArgs&, int, int, dim3, hipStream_t, hipError_t*) {
  return false;
}
constexpr long long tune_beam4_resident_for(int, int) { return 0; }
inline bool tune_beam_occupancy(int, int, int*, hipError_t*) { return false; }
inline unsigned* tune_steal_counters(size_t) { return nullptr; }
#endif

}  // namespace llm
