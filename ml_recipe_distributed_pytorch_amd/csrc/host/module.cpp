// pybind11 module _hq_host: native host runtime (batch synthesiser, CRC32C, WordPiece/BPE tokenizers).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "hq_host.h"

namespace py = pybind11;

void hq_register_tokenizers(py::module_& m);

PYBIND11_MODULE(_hq_host, m) {
  m.doc() = "Native host runtime for ml_recipe_distributed_pytorch_amd";
  m.def(
      "synth_dummy",
      [](int64_t ids, int64_t tt, int64_t mask, int B, int L, int q, int64_t vocab, int64_t pad, int64_t unk, int64_t cls,
         int64_t sep, bool bert_types, uint64_t seed, int threads) {
        if (q + 2 >= L) throw std::invalid_argument("max_question_len too large for max_seq_len");
        py::gil_scoped_release nogil;
        hq_synth_dummy(reinterpret_cast<int64_t*>(ids), reinterpret_cast<int64_t*>(tt), reinterpret_cast<bool*>(mask), B,
                       L, q, vocab, pad, unk, cls, sep, bert_types, seed, threads);
      },
      "Fill [B,L] int64 ids / token types / bool mask of dummy QA samples at the given addresses");
  m.def("crc32c", [](py::bytes data) {
    std::string s = data;
    return hq_crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  hq_register_tokenizers(m);
}
