// nc_span.h — layout of the per-context kernel-span buffer (nc_prof.cpp, nc_device.h).
#pragma once
namespace nc {
constexpr int kSpanCap = 4096;     // profiled launches between two span reads
constexpr int kSpanLines = 64;     // (start, end) slots per launch, one 128-byte line each
constexpr int kSpanStride = 16;    // u64 per line
constexpr int kSpanEdge = 8192;    // only the first / last kSpanEdge workgroups of a grid record
}
