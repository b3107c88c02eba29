// instantiation unit of the fused decode mat-vec for KT_IQ2_XXS / KT_IQ2_XS / KT_IQ2_S (see gemv_dec_impl.h)
#include "gemv_dec_impl.h"
template int dispatch_mode<KT_IQ2_XXS>(const DecArgs &, int, int, int, hipStream_t);
template int dispatch_mode<KT_IQ2_XS>(const DecArgs &, int, int, int, hipStream_t);
template int dispatch_mode<KT_IQ2_S>(const DecArgs &, int, int, int, hipStream_t);
