// Wide-row instantiations for configurable scoring resources (qs_kernels_res.inc).
#define QS_RES_WIDE 1
#include "qs_kernels_res.inc"
