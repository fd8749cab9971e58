// Internal interface between msda.hip (dispatch, workspace sizing) and msda_win.hip (the
// row-block MFMA backward for 16-bit values, D = 64).  Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

struct WinShape {
  long long B, S, M, Lq;
  int L, P;
  int T[16], start[16];
  int blk0[17];  // first row block of each level (set by msda_win_backward)
  int nblk;      // row blocks over all levels (set by msda_win_backward)
  int ntile;     // query tiles (set by msda_win_backward)
};

__attribute__((visibility("hidden"))) size_t msda_win_workspace_bytes(long long B, long long M, long long L,
                                                                     long long Lq);
__attribute__((visibility("hidden"))) int msda_win_supported(int value_dtype_is_bf16, long long D, long long P, long long Lq,
                                                                  long long row_floats);
__attribute__((visibility("hidden"))) int msda_win_backward(const void* value, const void* loc, const void* aw,
                                                            const void* gout, void* gval, void* gloc, void* gaw,
                                                            void* workspace, const WinShape* shape, int zeros,
                                                            hipStream_t st);
