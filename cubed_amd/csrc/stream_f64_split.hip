// stream_f64_split.hip -- the streaming kernels (stream_impl.h) for double values, split variant.
#define CUBED_STREAM_V double
#define CUBED_STREAM_SPLIT true
#include "stream_impl.h"
