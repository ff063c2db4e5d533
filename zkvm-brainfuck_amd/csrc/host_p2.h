// Host Poseidon2KoalaBear<16> permutation (host_p2.cpp): AVX-512 when the CPU has it, the
// scalar poseidon2_permute otherwise; bit-identical either way.
#pragma once
#include <cstdint>

namespace bfz {
void host_permute(uint32_t s[16]);
}
