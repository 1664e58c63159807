// Kubernetes resource.Quantity parsing.
//
// Pod gpu-mem limits are Quantities; the reference sums them with
// Quantity.Value() (pkg/utils/pod.go:146-155), which rounds UP to an integer
// (vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go:693-695).  This is
// an exact integer implementation of that contract for the three suffix
// families (binary SI, decimal SI, decimal exponent).
#pragma once

#include <cstdint>
#include <string_view>

namespace gsx {

// Parses a quantity string and returns ceil(value) saturated to int64.
// Returns false for malformed input.
bool parse_quantity(std::string_view s, int64_t* out);

// Go strconv.Atoi semantics on annotation values (no whitespace, optional
// sign, decimal digits, range-checked).  Returns false on any error.
bool parse_atoi(std::string_view s, int64_t* out);

}  // namespace gsx
