// instantiation unit of the fused decode mat-vec for KT_IQ3_XXS / KT_IQ3_S / KT_IQ1_S / KT_IQ1_M (see gemv_dec_impl.h)
#include "gemv_dec_impl.h"
template int dispatch_mode<KT_IQ3_XXS>(const DecArgs &, int, int, int, hipStream_t);
template int dispatch_mode<KT_IQ3_S>(const DecArgs &, int, int, int, hipStream_t);
template int dispatch_mode<KT_IQ1_S>(const DecArgs &, int, int, int, hipStream_t);
template int dispatch_mode<KT_IQ1_M>(const DecArgs &, int, int, int, hipStream_t);
