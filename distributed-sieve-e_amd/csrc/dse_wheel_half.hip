// dse_wheel_half.hip -- the wheel kernel again with half-size segments (2^16
// periods per plane, a 64 KiB LDS image) for the tails of ranges
// (launch_wheel_range_half, dse_internal.h): a range's last partial round of
// full segments is sieved as twice as many half segments, so more CUs share
// it. Same source as dse_wheel.hip; only the geometry differs.
#define DSE_WHEEL_LOG_KP 16
#define DSE_WHEEL_HALF_TU 1
#include "dse_wheel.hip"
