// dse_wheel_plain.hip -- the wheel kernel's instantiation for ranges without
// bucketed primes (N up to 1.1e12, the headline configs), in a translation unit
// of its own so it gets its own compile flags (Makefile: the default machine
// scheduler, under which its unit loop spills 13 SGPRs instead of 25 and runs
// 1.1% faster; the bucket instantiation in dse_wheel.hip keeps iterative-ILP).
// Same source as dse_wheel.hip; only launch_wheel_plain is emitted.
#define DSE_WHEEL_PLAIN_TU 1
#include "dse_wheel.hip"
