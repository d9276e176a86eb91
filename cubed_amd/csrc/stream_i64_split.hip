// stream_i64_split.hip -- the streaming kernels (stream_impl.h) for int64_t values, split variant.
#define CUBED_STREAM_V int64_t
#define CUBED_STREAM_SPLIT true
#include "stream_impl.h"
