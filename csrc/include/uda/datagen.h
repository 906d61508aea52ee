// Native generators of sorted map-output runs (see csrc/engine/datagen.cc).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace uda {
// result[map][reducer] = IFile partition stream (sorted records + EOF marker).
std::vector<std::vector<std::vector<uint8_t>>> generate_runs(const std::string& kind, int maps, int reducers,
                                                             int64_t rows_per_map, uint64_t seed);
}  // namespace uda
