// fedagg_k4.hip — reduce_kernel instantiations of libfedagg.so (see
// reduce_impl.h): one share of the (U, B) launcher set, compiled in
// parallel with the other units.
#include "reduce_impl.h"

FA_K_LAUNCH_U(, 4, 8)
FA_K_LAUNCH_CHAIN(, 4, 8)
