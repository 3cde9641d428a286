// Native tokenizers (replacing the Rust HF `tokenizers` the reference depends on):
//
// * WordPiece (BERT): BertNormalizer (clean text, CJK spacing, NFD accent strip, lowercase) +
//   BertPreTokenizer (split on whitespace and punctuation) + greedy longest-match-first WordPiece
//   with "##" continuations and max 100 chars per word.  No special tokens are added here; the
//   Python wrapper adds [CLS]/[SEP] only in legacy mode (reference quirk D11).
// * Byte-level BPE (RoBERTa): GPT-2 pre-tokenizer (contractions / ?\p{L}+ / ?\p{N}+ /
//   ?[^\s\p{L}\p{N}]+ / \s+(?!\S) / \s+), byte→unicode mapping, rank-ordered merges with optional
//   BPE-dropout, per-word cache when dropout is off.
// Unicode classes come from unicode_tables.inc generated out of Python's unicodedata.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <fstream>
#include <mutex>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "unicode_tables.inc"

namespace py = pybind11;

namespace {

bool in_ranges(uint32_t cp, const uint32_t (*r)[2], size_t n) {
  size_t lo = 0, hi = n;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (cp < r[mid][0]) hi = mid;
    else if (cp > r[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}

bool is_punct_bert(uint32_t c) {
  if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126)) return true;
  return in_ranges(c, kPunct, kPunct_n);
}
bool is_whitespace(uint32_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || in_ranges(c, kSpace, kSpace_n);
}
bool is_control(uint32_t c) {
  if (c == '\t' || c == '\n' || c == '\r') return false;
  return in_ranges(c, kControl, kControl_n);
}
bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) || (c >= 0x20000 && c <= 0x2A6DF) ||
         (c >= 0x2A700 && c <= 0x2B73F) || (c >= 0x2B740 && c <= 0x2B81F) || (c >= 0x2B820 && c <= 0x2CEAF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}
bool is_letter(uint32_t c) { return in_ranges(c, kLetter, kLetter_n); }
bool is_number(uint32_t c) { return in_ranges(c, kNumber, kNumber_n); }
bool is_mn(uint32_t c) { return in_ranges(c, kMn, kMn_n); }

uint32_t to_lower(uint32_t c) {
  if (c < 128) return (c >= 'A' && c <= 'Z') ? c + 32 : c;
  size_t lo = 0, hi = kLower_n;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (kLower[mid][0] < c) lo = mid + 1;
    else hi = mid;
  }
  return (lo < kLower_n && kLower[lo][0] == c) ? kLower[lo][1] : c;
}

void nfd_append(uint32_t c, std::vector<uint32_t>& out) {
  if (c < 0xC0) { out.push_back(c); return; }
  size_t lo = 0, hi = kNfdIndex_n;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (kNfdIndex[mid][0] < c) lo = mid + 1;
    else hi = mid;
  }
  if (lo < kNfdIndex_n && kNfdIndex[lo][0] == c) {
    for (uint32_t i = 0; i < kNfdIndex[lo][2]; ++i) out.push_back(kNfdData[kNfdIndex[lo][1] + i]);
  } else {
    out.push_back(c);
  }
}

std::vector<uint32_t> utf8_decode(const std::string& s) {
  std::vector<uint32_t> out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    const unsigned char c = s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
    else { out.push_back(0xFFFD); ++i; continue; }
    if (i + n > s.size()) { out.push_back(0xFFFD); break; }
    for (int k = 1; k < n; ++k) cp = (cp << 6) | (s[i + k] & 0x3F);
    out.push_back(cp);
    i += n;
  }
  return out;
}

void utf8_append(uint32_t cp, std::string& out) {
  if (cp < 0x80) out.push_back((char)cp);
  else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12))); out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18))); out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

std::string utf8_encode(const std::vector<uint32_t>& cps, size_t a, size_t b) {
  std::string out;
  for (size_t i = a; i < b; ++i) utf8_append(cps[i], out);
  return out;
}

// =========================================================================================== WordPiece
class WordPiece {
 public:
  WordPiece(const std::string& vocab_file, bool lowercase, int strip_accents, bool handle_chinese_chars,
            const std::string& unk, int max_chars)
      : lowercase_(lowercase), strip_(strip_accents < 0 ? lowercase : strip_accents != 0),
        cjk_(handle_chinese_chars), max_chars_(max_chars) {
    std::ifstream f(vocab_file);
    if (!f) throw std::runtime_error("cannot open vocab file " + vocab_file);
    std::string line;
    while (std::getline(f, line)) {
      while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
      if (!vocab_.count(line)) vocab_[line] = (int)inv_.size();
      inv_.push_back(line);
    }
    auto it = vocab_.find(unk);
    unk_id_ = it == vocab_.end() ? -1 : it->second;
  }

  // BertNormalizer + BertPreTokenizer
  std::vector<std::vector<uint32_t>> pre_tokenize(const std::string& text) const {
    std::vector<uint32_t> cps = utf8_decode(text), norm;
    norm.reserve(cps.size() + 16);
    for (uint32_t c : cps) {
      if (c == 0 || c == 0xFFFD || is_control(c)) continue;
      if (is_whitespace(c)) { norm.push_back(' '); continue; }
      if (cjk_ && is_cjk(c)) { norm.push_back(' '); norm.push_back(c); norm.push_back(' '); continue; }
      norm.push_back(c);
    }
    if (strip_) {
      std::vector<uint32_t> tmp;
      tmp.reserve(norm.size());
      for (uint32_t c : norm) {
        const size_t before = tmp.size();
        nfd_append(c, tmp);
        size_t w = before;
        for (size_t i = before; i < tmp.size(); ++i)
          if (!is_mn(tmp[i])) tmp[w++] = tmp[i];
        tmp.resize(w);
      }
      norm.swap(tmp);
    }
    if (lowercase_) {
      std::vector<uint32_t> tmp;
      tmp.reserve(norm.size());
      for (uint32_t c : norm) {
        if (c == 0x130) { tmp.push_back('i'); tmp.push_back(0x307); continue; }  // the one multi-char lower
        tmp.push_back(to_lower(c));
      }
      norm.swap(tmp);
    }
    std::vector<std::vector<uint32_t>> words;
    std::vector<uint32_t> cur;
    for (uint32_t c : norm) {
      if (is_whitespace(c)) {
        if (!cur.empty()) { words.push_back(cur); cur.clear(); }
      } else if (is_punct_bert(c)) {
        if (!cur.empty()) { words.push_back(cur); cur.clear(); }
        words.push_back({c});
      } else {
        cur.push_back(c);
      }
    }
    if (!cur.empty()) words.push_back(cur);
    return words;
  }

  void wordpiece(const std::vector<uint32_t>& w, std::vector<int>& out) const {
    if ((int)w.size() > max_chars_) { out.push_back(unk_id_); return; }
    std::vector<int> pieces;
    size_t start = 0;
    while (start < w.size()) {
      size_t end = w.size();
      int found = -1;
      while (start < end) {
        std::string sub = start > 0 ? "##" : "";
        sub += utf8_encode(w, start, end);
        auto it = vocab_.find(sub);
        if (it != vocab_.end()) { found = it->second; break; }
        --end;
      }
      if (found < 0) { out.push_back(unk_id_); return; }
      pieces.push_back(found);
      start = end;
    }
    out.insert(out.end(), pieces.begin(), pieces.end());
  }

  std::vector<int> encode(const std::string& text) const {
    std::vector<int> out;
    for (const auto& w : pre_tokenize(text)) wordpiece(w, out);
    return out;
  }

  std::vector<std::string> tokenize(const std::string& text) const {
    std::vector<std::string> out;
    for (int id : encode(text)) out.push_back(id >= 0 && id < (int)inv_.size() ? inv_[id] : "[UNK]");
    return out;
  }

  int token_to_id(const std::string& t) const {
    auto it = vocab_.find(t);
    return it == vocab_.end() ? -1 : it->second;
  }
  std::string id_to_token(int id) const { return id >= 0 && id < (int)inv_.size() ? inv_[id] : ""; }
  size_t size() const { return inv_.size(); }

 private:
  std::unordered_map<std::string, int> vocab_;
  std::vector<std::string> inv_;
  bool lowercase_, strip_, cjk_;
  int max_chars_;
  int unk_id_ = -1;
};

// ======================================================================================= byte-level BPE
class ByteLevelBPE {
 public:
  ByteLevelBPE(const std::string& vocab_json, const std::string& merges_txt, double dropout, uint64_t seed)
      : dropout_(dropout), rng_(seed) {
    // byte → printable unicode (GPT-2 bytes_to_unicode)
    std::vector<int> bs;
    for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
    for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
    for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
    std::vector<int> cs(bs);
    int n = 0;
    for (int b = 0; b < 256; ++b) {
      if (std::find(bs.begin(), bs.end(), b) == bs.end()) { bs.push_back(b); cs.push_back(256 + n++); }
    }
    for (size_t i = 0; i < bs.size(); ++i) {
      byte2u_[bs[i]] = (uint32_t)cs[i];
      u2byte_[(uint32_t)cs[i]] = (uint8_t)bs[i];
    }
    load_vocab(vocab_json);
    std::ifstream f(merges_txt);
    if (!f) throw std::runtime_error("cannot open merges file " + merges_txt);
    std::string line;
    int rank = 0;
    while (std::getline(f, line)) {
      while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
      if (line.empty() || line.rfind("#version", 0) == 0) continue;
      const size_t sp = line.find(' ');
      if (sp == std::string::npos) continue;
      ranks_[line.substr(0, sp) + "\x01" + line.substr(sp + 1)] = rank++;
    }
  }

  std::vector<int> encode(const std::string& text) {
    std::vector<int> out;
    for (const std::string& piece : pre_tokenize(text)) {
      if (dropout_ <= 0) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = cache_.find(piece);
        if (it != cache_.end()) { out.insert(out.end(), it->second.begin(), it->second.end()); continue; }
      }
      std::vector<int> ids = bpe(piece);
      if (dropout_ <= 0) {
        std::lock_guard<std::mutex> g(mu_);
        if (cache_.size() < 200000) cache_[piece] = ids;
      }
      out.insert(out.end(), ids.begin(), ids.end());
    }
    return out;
  }

  std::string decode(const std::vector<int>& ids) const {
    std::string bytes;
    for (int id : ids) {
      if (id < 0 || id >= (int)inv_.size()) continue;
      for (uint32_t cp : utf8_decode(inv_[id])) {
        auto it = u2byte_.find(cp);
        if (it != u2byte_.end()) bytes.push_back((char)it->second);
      }
    }
    return bytes;
  }

  int token_to_id(const std::string& t) const {
    auto it = vocab_.find(t);
    return it == vocab_.end() ? -1 : it->second;
  }
  size_t size() const { return inv_.size(); }

 private:
  void load_vocab(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open vocab file " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string s = ss.str();
    // minimal JSON object parser: {"token": id, ...} with \uXXXX / \" / \\ escapes
    size_t i = s.find('{');
    if (i == std::string::npos) throw std::runtime_error("bad vocab json");
    ++i;
    int max_id = -1;
    std::vector<std::pair<std::string, int>> items;
    while (i < s.size()) {
      while (i < s.size() && (isspace((unsigned char)s[i]) || s[i] == ',')) ++i;
      if (i >= s.size() || s[i] == '}') break;
      if (s[i] != '"') throw std::runtime_error("bad vocab json key");
      ++i;
      std::string key;
      while (i < s.size() && s[i] != '"') {
        if (s[i] == '\\') {
          ++i;
          const char e = s[i];
          if (e == 'u') {
            uint32_t cp = std::stoul(s.substr(i + 1, 4), nullptr, 16);
            i += 4;
            if (cp >= 0xD800 && cp <= 0xDBFF && s[i + 1] == '\\' && s[i + 2] == 'u') {
              const uint32_t lo = std::stoul(s.substr(i + 3, 4), nullptr, 16);
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              i += 6;
            }
            utf8_append(cp, key);
          } else if (e == 'n') key.push_back('\n');
          else if (e == 't') key.push_back('\t');
          else if (e == 'r') key.push_back('\r');
          else if (e == 'b') key.push_back('\b');
          else if (e == 'f') key.push_back('\f');
          else key.push_back(e);
          ++i;
        } else {
          key.push_back(s[i++]);
        }
      }
      ++i;
      while (i < s.size() && (isspace((unsigned char)s[i]) || s[i] == ':')) ++i;
      size_t j = i;
      while (j < s.size() && (isdigit((unsigned char)s[j]) || s[j] == '-')) ++j;
      const int id = std::stoi(s.substr(i, j - i));
      i = j;
      items.emplace_back(key, id);
      max_id = std::max(max_id, id);
    }
    inv_.assign(max_id + 1, "");
    for (auto& kv : items) { vocab_[kv.first] = kv.second; inv_[kv.second] = kv.first; }
  }

  // GPT-2 pattern: 's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
  std::vector<std::string> pre_tokenize(const std::string& text) const {
    std::vector<uint32_t> c = utf8_decode(text);
    std::vector<std::string> out;
    const size_t n = c.size();
    size_t i = 0;
    auto ws = [&](size_t k) { return k < n && is_whitespace(c[k]); };
    while (i < n) {
      size_t j = i;
      if (c[i] == '\'' && i + 1 < n) {
        const uint32_t a = c[i + 1], b = i + 2 < n ? c[i + 2] : 0;
        if (a == 's' || a == 't' || a == 'm' || a == 'd') j = i + 2;
        else if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) j = i + 3;
      }
      if (j == i) {
        size_t k = i;
        if (c[k] == ' ' && k + 1 < n && !is_whitespace(c[k + 1])) ++k;
        if (k < n && is_letter(c[k])) {
          while (k < n && is_letter(c[k])) ++k;
          j = k;
        } else if (k < n && is_number(c[k])) {
          while (k < n && is_number(c[k])) ++k;
          j = k;
        } else if (k < n && !is_whitespace(c[k])) {
          while (k < n && !is_whitespace(c[k]) && !is_letter(c[k]) && !is_number(c[k])) ++k;
          j = k;
        } else {
          // whitespace run: \s+(?!\S) keeps the last space for the next word
          size_t e = i;
          while (ws(e)) ++e;
          j = (e < n && e - i > 1) ? e - 1 : e;
          if (j == i) j = i + 1;
        }
      }
      out.push_back(utf8_encode(c, i, j));
      i = j;
    }
    return out;
  }

  std::vector<int> bpe(const std::string& piece) {
    std::vector<std::string> sym;
    for (unsigned char b : piece) {
      std::string u;
      utf8_append(byte2u_[b], u);
      sym.push_back(u);
    }
    std::uniform_real_distribution<double> uni(0.0, 1.0);
    while (sym.size() > 1) {
      int best = -1, best_rank = INT32_MAX;
      for (size_t k = 0; k + 1 < sym.size(); ++k) {
        auto it = ranks_.find(sym[k] + "\x01" + sym[k + 1]);
        if (it == ranks_.end()) continue;
        if (dropout_ > 0 && uni(rng_) < dropout_) continue;
        if (it->second < best_rank) { best_rank = it->second; best = (int)k; }
      }
      if (best < 0) break;
      const std::string a = sym[best], b = sym[best + 1];
      std::vector<std::string> merged;
      for (size_t k = 0; k < sym.size(); ++k) {
        if (k + 1 < sym.size() && sym[k] == a && sym[k + 1] == b) { merged.push_back(a + b); ++k; }
        else merged.push_back(sym[k]);
      }
      sym.swap(merged);
    }
    std::vector<int> ids;
    for (auto& s : sym) {
      auto it = vocab_.find(s);
      if (it != vocab_.end()) ids.push_back(it->second);
    }
    return ids;
  }

  double dropout_;
  std::mt19937_64 rng_;
  std::unordered_map<uint8_t, uint32_t> byte2u_;
  std::unordered_map<uint32_t, uint8_t> u2byte_;
  std::unordered_map<std::string, int> vocab_, ranks_;
  std::vector<std::string> inv_;
  std::unordered_map<std::string, std::vector<int>> cache_;
  std::mutex mu_;
};

}  // namespace

void hq_register_tokenizers(py::module_& m) {
  py::class_<WordPiece>(m, "WordPiece")
      .def(py::init<const std::string&, bool, int, bool, const std::string&, int>(), py::arg("vocab_file"),
           py::arg("lowercase") = true, py::arg("strip_accents") = -1, py::arg("handle_chinese_chars") = true,
           py::arg("unk_token") = "[UNK]", py::arg("max_input_chars_per_word") = 100)
      .def("encode", &WordPiece::encode, py::call_guard<py::gil_scoped_release>())
      .def("encode_batch",
           [](const WordPiece& w, const std::vector<std::string>& texts) {
             std::vector<std::vector<int>> out(texts.size());
             py::gil_scoped_release nogil;
             for (size_t i = 0; i < texts.size(); ++i) out[i] = w.encode(texts[i]);
             return out;
           })
      .def("tokenize", &WordPiece::tokenize)
      .def("token_to_id", &WordPiece::token_to_id)
      .def("id_to_token", &WordPiece::id_to_token)
      .def("__len__", &WordPiece::size);
  py::class_<ByteLevelBPE>(m, "ByteLevelBPE")
      .def(py::init<const std::string&, const std::string&, double, uint64_t>(), py::arg("vocab_file"),
           py::arg("merges_file"), py::arg("dropout") = 0.0, py::arg("seed") = 0)
      .def("encode", &ByteLevelBPE::encode)
      .def("decode", &ByteLevelBPE::decode)
      .def("token_to_id", &ByteLevelBPE::token_to_id)
      .def("__len__", &ByteLevelBPE::size);
}
