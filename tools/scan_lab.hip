// Scan-kernel A/B lab (development tool, not part of the product ABI).
// Includes the product source so every variant is the exact production code,
// and exports one entry point that launches a chosen scan variant.
#include "../hybrid-rag-colbertv2_amd/csrc/colbert_mi355x.hip"

extern "C" int lab_scan(cbv2_index* ix, int variant, const void* Q, int B, int lq, float* out, int64_t ld,
                        void* stream) {
  return scan_maxsim(ix, (const uint16_t*)Q, B, lq, out, ld, (hipStream_t)stream, variant);
}
