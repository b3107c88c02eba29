// instantiation unit of the fused decode mat-vec for KT_Q2_K (see gemv_dec_impl.h)
#include "gemv_dec_impl.h"
template int dispatch_mode<KT_Q2_K>(const DecArgs &, int, int, int, hipStream_t);
