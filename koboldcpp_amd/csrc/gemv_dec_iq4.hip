// instantiation unit of the fused decode mat-vec for KT_IQ4_NL / KT_IQ4_XS (see gemv_dec_impl.h)
#include "gemv_dec_impl.h"
template int dispatch_mode<KT_IQ4_NL>(const DecArgs &, int, int, int, hipStream_t);
template int dispatch_mode<KT_IQ4_XS>(const DecArgs &, int, int, int, hipStream_t);
