// stream_f64.hip -- the streaming kernels (stream_impl.h) for double values.
#define CUBED_STREAM_V double
#define CUBED_STREAM_SPLIT false
#include "stream_impl.h"
