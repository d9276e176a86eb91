// stream_i64.hip -- the streaming kernels (stream_impl.h) for int64_t values.
#define CUBED_STREAM_V int64_t
#define CUBED_STREAM_SPLIT false
#include "stream_impl.h"
