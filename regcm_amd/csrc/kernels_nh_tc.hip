// kernels_nh_tc.hip -- k_nh_tend_c (kernels_nh.hip) in a translation unit of its own, compiled
// with the device scheduler the Makefile names for it (SCHED_kernels_nh_tc)
#define RCM_NH_TEND_C_TU
#include "kernels_nh.hip"
