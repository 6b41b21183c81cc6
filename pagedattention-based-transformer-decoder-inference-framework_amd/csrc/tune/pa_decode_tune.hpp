// Tuning build only: the experiment kernels of csrc/tune/pa_decode_tune.hip
// that pa_decode.hip launches when LLM_BEAM4 / LLM_BEAM_MFMA switch them on.
#pragma once

#include "pa_split.hpp"

namespace llm {

// resident waves of pa_beam4_kernel over the chip (0: shape not supported)
long long tune_beam4_resident_for(int D, int TS);
// pa_beam4_kernel over the launch's (group, head, split) waves
hipError_t tune_launch_beam4(const PaSplitArgs& a, int D, int TS, hipStream_t st);
// pa_beam_mfma_kernel (D 128, page 16) on pa_split_kernel's BEAM grid
hipError_t tune_launch_beam_mfma(const PaSplitArgs& a, dim3 grid, hipStream_t st);
hipError_t tune_beam_mfma_occupancy(int* blocks);
// the shipped BEAM form of pa_split_kernel (D 128, page 16) with a trivial
// consumer (LOAD_ONLY): its loads, LDS staging and barriers without the maths
hipError_t tune_launch_beam_loads_only(const PaSplitArgs& a, dim3 grid, hipStream_t st);
// the same form with the shared chunks delivered by an LDS-DMA ring of `ring`
// chunks (pa_split_kernel RING), optionally with the trivial consumer
// the shipped form with per-wave timestamps (STAMPS; pa_tune_stamps copies them)
hipError_t tune_launch_beam_stamps(const PaSplitArgs& a, dim3 grid, hipStream_t st);
// the decoder's steal form with per-wave stamps (pa_tune_stamps8 copies them)
hipError_t tune_launch_steal_stamps(const PaSplitArgs& a, dim3 grid, hipStream_t st);
hipError_t tune_launch_beam_ring(const PaSplitArgs& a, dim3 grid, hipStream_t st, int ring,
                                 bool load_only);

}  // namespace llm
