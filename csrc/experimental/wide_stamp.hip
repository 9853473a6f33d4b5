// Probe build of the wide mid-M GEMM (csrc/kernels/wide_gemm.hip) with per-block wall-clock
// stamps at its phase boundaries (bench/wide_stamp_probe.py).  The production kernel is the
// same source; WIDE_STAMP only adds the stores of the stamps.  Entry points are renamed so
// the experimental library never shadows the kernel library's.
#define WIDE_STAMP 1
#define p2p_wide_dispatch p2p_wide_stamp_dispatch
#define p2p_wide_split_fault p2p_wide_stamp_split_fault
#define p2p_wide_resident p2p_wide_stamp_resident
#define p2p_wide_max_split p2p_wide_stamp_max_split
#include "../kernels/wide_gemm.hip"
