// WordCounter: the wordfreq map with in-mapper combining (kernels in
// csrc/kernels/wordcount.hip). Feed it text chunks with add(); finish()
// returns KV(word+NUL, int32 count) with one pair per distinct word — the
// same pairs MR-MPI's map(read_words) + compress(count) would leave
// (reference oink/map_read_words.cpp:14-30, src/mapreduce.cpp:749-851),
// without ever materialising one KV per word occurrence.
#pragma once
#include <string>
#include <unordered_map>

#include "kv.h"

namespace mrh {

class WordCounter {
 public:
  explicit WordCounter(at::Device dev, int64_t init_slots = 1 << 20);
  // count the words of text[0, n) (buffer padded by >= 32 bytes, n < 2^31)
  void add(const at::Tensor& text, int64_t n);
  // (word+NUL, int32 count) pairs; the counter is reset afterwards
  KV finish();
  int64_t words() const { return words_; }   // occurrences added so far
  int64_t capacity() const { return cap_; }  // device table slots

 private:
  void reserve(int64_t used, int64_t new_words, int64_t new_bytes);

  at::Device dev_;
  int64_t cap_ = 0, init_ = 0, words_ = 0, used_ = 0, arena_used_ = 0;
  at::Tensor slots_, counts_, arena_, ctr_;
  std::unordered_map<std::string, int64_t> host_;  // CPU engine
};

}  // namespace mrh
