// stream_f32.hip -- the streaming kernels (stream_impl.h) for float values.
#define CUBED_STREAM_V float
#define CUBED_STREAM_SPLIT false
#include "stream_impl.h"
