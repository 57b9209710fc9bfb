// decode_local256_any.hip -- the local decode on 256-byte row runs for sub-chunks that are not
// multiples of 8 (k_stream_local256<..., ANY = true>): decode_local256.hip built as its own
// translation unit (compiles in parallel with the 8-byte-row instantiations).
#define LOCAL256_ANY 1
#include "decode_local256.hip"
