/* cbf_amd measurement hooks: NOT part of the drop-in surface (include/cbf_amd.h).
 *
 * bench.py and the GPU tests time the dominant kernel of a lattice timestep through these: the
 * same advance as the public calls, with the filter kernel's own start / end (or its end on the
 * stream) recorded into caller-supplied events, and a query of where a window's full QPs are
 * solved (the label of a bench line).  Results are bit-identical to the public calls'
 * (tests/test_gpu_window.py::test_timed_advance_equals_marked,
 * tests/test_gpu_parity.py::test_lattice_advance_marked_equals_advance). */
#ifndef CBF_AMD_MEASURE_H
#define CBF_AMD_MEASURE_H

#include "cbf_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cbf_lattice_window_advance with the filter kernel launched so that filter_start / filter_stop
 * (hipEvent_t, both required, created beforehand) carry that dispatch's own start and end times
 * (hipExtLaunchKernel): the bench's measurement of the dominant kernel, free of the launch's
 * dispatch and end-of-kernel cache flush, as a kernel trace measures it.  (ABI 6) */
int cbf_lattice_window_advance_timed(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H,
                                     const double* pos, double T, double* pos_out, double* u, int32_t* status,
                                     int32_t* nbr_count, uint64_t* stats, void* workspace, size_t workspace_bytes,
                                     void* filter_start, void* filter_stop, void* stream);
/* cbf_lattice_advance, recording `filter_done` (a hipEvent_t, nullable) on `stream` between the
 * filter kernel and the queued-QP kernel: the measurement hook for the dominant kernel alone. */
int cbf_lattice_advance_marked(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                               int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double T,
                               double* pos_out, double* u, int32_t* status, int32_t* nbr_count, int32_t guard_rows,
                               double* extents, uint64_t* solves, void* workspace, size_t workspace_bytes,
                               void* filter_done, void* stream);
/* cbf_lattice_advance with the filter's own start / end times in filter_start / filter_stop (as
 * cbf_lattice_window_advance_timed).  (ABI 6) */
int cbf_lattice_advance_timed(const cbf_params* p, const cbf_grid* grid, int32_t W, int32_t H, int32_t row_begin,
                              int32_t row_end, int32_t win_row0, int32_t win_rows, const double* pos, double T,
                              double* pos_out, double* u, int32_t* status, int32_t* nbr_count, int32_t guard_rows,
                              double* extents, uint64_t* solves, void* workspace, size_t workspace_bytes,
                              void* filter_start, void* filter_stop, void* stream);
/* 1 if a lattice window of n agents solves its full QPs inside the filter kernel under p
 * (cbf_params.solve_inline_max, < 0: the library's threshold), 0 if the queued-QP kernel does. */
int cbf_lattice_solves_inline(const cbf_params* p, int64_t n);

#ifdef __cplusplus
}
#endif

#endif /* CBF_AMD_MEASURE_H */
