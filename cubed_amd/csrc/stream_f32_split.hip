// stream_f32_split.hip -- the streaming kernels (stream_impl.h) for float values, split variant.
#define CUBED_STREAM_V float
#define CUBED_STREAM_SPLIT true
#include "stream_impl.h"
