// instantiation unit of the fused decode mat-vec for KT_Q4_K (see gemv_dec_impl.h)
#include "gemv_dec_impl.h"
template int dispatch_mode<KT_Q4_K>(const DecArgs &, int, int, int, hipStream_t);
