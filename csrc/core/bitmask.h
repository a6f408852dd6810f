// Partition bitmask (cpumask_t analog). Up to 256 execution partitions
// (32 GPUs x 8 XCDs) per engine.  Semantics of cycle()/first() follow
// the cpumask helpers the reference scheduler relies on
// (X:xen/include/xen/cpumask.h: cpumask_cycle wraps past the end).
#pragma once
#include <cstdint>
#include <string>

namespace gpbs {

constexpr int kMaxPartitions = 256;

struct Mask {
  uint64_t w[kMaxPartitions / 64] = {0, 0, 0, 0};

  static Mask none() { return Mask{}; }
  static Mask all(int n) {
    Mask m;
    for (int i = 0; i < n; ++i) m.set(i);
    return m;
  }
  static Mask of(int i) {
    Mask m;
    m.set(i);
    return m;
  }
  void set(int i) { w[i >> 6] |= (1ull << (i & 63)); }
  void clear(int i) { w[i >> 6] &= ~(1ull << (i & 63)); }
  bool test(int i) const { return i >= 0 && i < kMaxPartitions && ((w[i >> 6] >> (i & 63)) & 1); }
  bool empty() const { return !(w[0] | w[1] | w[2] | w[3]); }
  int weight() const {
    int c = 0;
    for (auto x : w) c += __builtin_popcountll(x);
    return c;
  }
  Mask operator&(const Mask& o) const {
    Mask m;
    for (int i = 0; i < 4; ++i) m.w[i] = w[i] & o.w[i];
    return m;
  }
  Mask operator|(const Mask& o) const {
    Mask m;
    for (int i = 0; i < 4; ++i) m.w[i] = w[i] | o.w[i];
    return m;
  }
  Mask andnot(const Mask& o) const {
    Mask m;
    for (int i = 0; i < 4; ++i) m.w[i] = w[i] & ~o.w[i];
    return m;
  }
  bool operator==(const Mask& o) const {
    for (int i = 0; i < 4; ++i)
      if (w[i] != o.w[i]) return false;
    return true;
  }
  // First set bit >= from, or -1.
  int next(int from) const {
    for (int i = from < 0 ? 0 : from; i < kMaxPartitions; ++i) {
      uint64_t word = w[i >> 6] >> (i & 63);
      if (word) return i + __builtin_ctzll(word);
      i |= 63;  // skip to end of word
    }
    return -1;
  }
  int first() const { return next(0); }
  // Next set bit strictly after n, wrapping around; -1 if empty.
  int cycle(int n) const {
    int r = next(n + 1);
    if (r < 0) r = next(0);
    return r;
  }
  std::string str() const {
    // Compact range list "0-3,6".
    std::string s;
    int i = first();
    while (i >= 0) {
      int j = i;
      while (test(j + 1)) ++j;
      if (!s.empty()) s += ",";
      s += std::to_string(i);
      if (j > i) s += "-" + std::to_string(j);
      i = next(j + 1);
    }
    return s.empty() ? "none" : s;
  }
};

}  // namespace gpbs
