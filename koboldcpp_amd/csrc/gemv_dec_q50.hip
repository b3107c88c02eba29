// instantiation unit of the fused decode mat-vec for KT_Q5_0 (see gemv_dec_impl.h)
#include "gemv_dec_impl.h"
template int dispatch_mode<KT_Q5_0>(const DecArgs &, int, int, int, hipStream_t);
