// dcor_rds.cpp -- R serialization (readRDS) reader for the HRS ingest path, no R needed.
//
// The reference reads its panel with readRDS("hrs_long_panel.rds") and keeps wave-2 complete
// cases of (agey_e, bmi) (real-data-sims.R:13, 38-41).  This is a self-contained reader of the
// format R writes there: gzip (zlib) around the XDR binary serialization, format version 2 or
// 3.  It decodes the object graph -- vectors, pairlists, symbols, references, attributes,
// compact ALTREP sequences -- into a small tree, and exposes a data.frame's columns by name.
// Input is untrusted: every length is bounds-checked against the buffer.
#include <zlib.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/dcor.h"

namespace {

enum : int {
  NILSXP = 0, SYMSXP = 1, LISTSXP = 2, CLOSXP = 3, ENVSXP = 4, PROMSXP = 5, LANGSXP = 6,
  CHARSXP = 9, LGLSXP = 10, INTSXP = 13, REALSXP = 14, CPLXSXP = 15, STRSXP = 16, DOTSXP = 17,
  VECSXP = 19, EXPRSXP = 20, RAWSXP = 24, S4SXP = 25,
  ALTREP_SXP = 238, ATTRLISTSXP = 239, ATTRLANGSXP = 240, BASEENV_SXP = 241, EMPTYENV_SXP = 242,
  GLOBALENV_SXP = 253, NILVALUE_SXP = 254, REFSXP = 255, UNBOUNDVALUE_SXP = 252,
  MISSINGARG_SXP = 251, BASENAMESPACE_SXP = 250
};
constexpr int32_t R_NA_INT = INT32_MIN;

struct Node;
using NodeP = std::shared_ptr<Node>;

struct Node {
  int type = NILSXP;
  std::vector<double> real;       // REALSXP (CPLX: interleaved)
  std::vector<int32_t> ints;      // INTSXP / LGLSXP
  std::vector<std::string> strs;  // STRSXP (na flags below); CHARSXP / SYMSXP name in strs[0]
  std::vector<uint8_t> str_na;
  std::vector<NodeP> items;       // VECSXP / EXPRSXP elements; pairlist CARs
  std::vector<NodeP> tags;        // pairlist TAGs (SYMSXP nodes or null)
  NodeP attr;                     // attribute pairlist
  int64_t length() const {
    switch (type) {
      case REALSXP: return (int64_t)real.size();
      case CPLXSXP: return (int64_t)real.size() / 2;
      case INTSXP: case LGLSXP: return (int64_t)ints.size();
      case STRSXP: return (int64_t)strs.size();
      case VECSXP: case EXPRSXP: case LISTSXP: return (int64_t)items.size();
      default: return 0;
    }
  }
  NodeP get_attr(const char* name) const {
    if (!attr) return nullptr;
    for (size_t i = 0; i < attr->items.size(); ++i)
      if (attr->tags[i] && !attr->tags[i]->strs.empty() && attr->tags[i]->strs[0] == name)
        return attr->items[i];
    return nullptr;
  }
};

struct ParseError {
  std::string msg;
};

class Reader {
 public:
  Reader(const unsigned char* p, size_t n) : p_(p), n_(n) {}
  NodeP parse() {
    need(2);
    if (!(p_[0] == 'X' && p_[1] == '\n'))
      throw ParseError{"not an XDR R serialization (expected 'X\\n'; ASCII and native formats are not supported)"};
    pos_ = 2;
    const int version = i32();
    (void)i32();  // writer R version
    (void)i32();  // minimal reader version
    if (version == 3) {
      const int nelen = i32();
      if (nelen < 0 || nelen > 4096) throw ParseError{"bad native-encoding length"};
      skip((size_t)nelen);
    } else if (version != 2) {
      throw ParseError{"unsupported serialization version " + std::to_string(version)};
    }
    return item(0);
  }

 private:
  const unsigned char* p_;
  size_t n_;
  size_t pos_ = 0;
  std::vector<NodeP> refs_;

  void need(size_t k) const {
    if (k > n_ || pos_ > n_ - k) throw ParseError{"truncated RDS stream"};
  }
  void skip(size_t k) { need(k); pos_ += k; }
  int32_t i32() {
    need(4);
    const uint32_t v = ((uint32_t)p_[pos_] << 24) | ((uint32_t)p_[pos_ + 1] << 16) |
                       ((uint32_t)p_[pos_ + 2] << 8) | (uint32_t)p_[pos_ + 3];
    pos_ += 4;
    return (int32_t)v;
  }
  double f64() {
    need(8);
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) v = (v << 8) | p_[pos_ + b];
    pos_ += 8;
    double d;
    std::memcpy(&d, &v, 8);
    return d;
  }
  int64_t vec_length() {
    const int32_t len = i32();
    if (len >= 0) return len;
    if (len != -1) throw ParseError{"bad vector length"};
    const uint32_t hi = (uint32_t)i32(), lo = (uint32_t)i32();  // long vector
    const int64_t l = ((int64_t)hi << 32) | lo;
    if (l < 0) throw ParseError{"bad long vector length"};
    return l;
  }
  void check_count(int64_t count, size_t elem) const {
    if (count < 0 || (uint64_t)count > (uint64_t)(n_ - pos_) / (elem ? elem : 1))
      throw ParseError{"vector longer than the stream"};
  }

  NodeP item(int depth) {
    if (depth > 4000) throw ParseError{"object nesting too deep"};
    const int32_t flags = i32();
    const int type = flags & 0xFF;
    const bool has_attr = (flags >> 9) & 1, has_tag = (flags >> 10) & 1;
    switch (type) {
      case NILVALUE_SXP: case EMPTYENV_SXP: case BASEENV_SXP: case GLOBALENV_SXP:
      case UNBOUNDVALUE_SXP: case MISSINGARG_SXP: case BASENAMESPACE_SXP:
        return std::make_shared<Node>();
      case REFSXP: {
        int idx = (flags >> 8);
        if (idx == 0) idx = i32();
        if (idx < 1 || (size_t)idx > refs_.size()) throw ParseError{"bad reference index"};
        return refs_[(size_t)idx - 1];
      }
      case SYMSXP: {
        auto s = std::make_shared<Node>();
        s->type = SYMSXP;
        refs_.push_back(s);
        NodeP name = item(depth + 1);
        s->strs.push_back(name->strs.empty() ? std::string() : name->strs[0]);
        return s;
      }
      case ENVSXP: {
        auto e = std::make_shared<Node>();
        e->type = ENVSXP;
        refs_.push_back(e);
        (void)i32();  // locked
        (void)item(depth + 1);  // enclos
        (void)item(depth + 1);  // frame
        (void)item(depth + 1);  // hashtab
        e->attr = item(depth + 1);
        return e;
      }
      case LISTSXP: case LANGSXP: case CLOSXP: case PROMSXP: case DOTSXP: case ATTRLISTSXP:
      case ATTRLANGSXP: {
        // pairlist: iterate along the CDR chain instead of recursing on it
        auto head = std::make_shared<Node>();
        head->type = LISTSXP;
        bool attr = has_attr, tag = has_tag;
        for (;;) {
          if (attr) (void)item(depth + 1);
          head->tags.push_back(tag ? item(depth + 1) : nullptr);
          head->items.push_back(item(depth + 1));
          const int32_t f2 = i32();
          const int t2 = f2 & 0xFF;
          if (t2 == NILVALUE_SXP) break;
          if (!(t2 == LISTSXP || t2 == LANGSXP || t2 == ATTRLISTSXP || t2 == ATTRLANGSXP ||
                t2 == DOTSXP)) {
            pos_ -= 4;  // a non-pairlist CDR: read it as one more element
            head->tags.push_back(nullptr);
            head->items.push_back(item(depth + 1));
            break;
          }
          attr = (f2 >> 9) & 1;
          tag = (f2 >> 10) & 1;
        }
        return head;
      }
      case CHARSXP: {
        auto c = std::make_shared<Node>();
        c->type = CHARSXP;
        const int32_t len = i32();
        if (len == -1) {
          c->strs.emplace_back();
          c->str_na.push_back(1);
        } else {
          if (len < 0) throw ParseError{"bad string length"};
          need((size_t)len);
          c->strs.emplace_back((const char*)p_ + pos_, (size_t)len);
          c->str_na.push_back(0);
          pos_ += (size_t)len;
        }
        return c;
      }
      case LGLSXP: case INTSXP: {
        auto v = std::make_shared<Node>();
        v->type = type;
        const int64_t len = vec_length();
        check_count(len, 4);
        v->ints.resize((size_t)len);
        for (int64_t i = 0; i < len; ++i) v->ints[(size_t)i] = i32();
        if (has_attr) v->attr = item(depth + 1);
        return v;
      }
      case REALSXP: case CPLXSXP: {
        auto v = std::make_shared<Node>();
        v->type = type;
        const int64_t len = vec_length() * (type == CPLXSXP ? 2 : 1);
        check_count(len, 8);
        v->real.resize((size_t)len);
        for (int64_t i = 0; i < len; ++i) v->real[(size_t)i] = f64();
        if (has_attr) v->attr = item(depth + 1);
        return v;
      }
      case RAWSXP: {
        auto v = std::make_shared<Node>();
        v->type = RAWSXP;
        const int64_t len = vec_length();
        check_count(len, 1);
        skip((size_t)len);
        if (has_attr) v->attr = item(depth + 1);
        return v;
      }
      case STRSXP: {
        auto v = std::make_shared<Node>();
        v->type = STRSXP;
        const int64_t len = vec_length();
        check_count(len, 4);
        v->strs.reserve((size_t)len);
        v->str_na.reserve((size_t)len);
        for (int64_t i = 0; i < len; ++i) {
          NodeP c = item(depth + 1);
          v->strs.push_back(c->strs.empty() ? std::string() : c->strs[0]);
          v->str_na.push_back(c->str_na.empty() ? 1 : c->str_na[0]);
        }
        if (has_attr) v->attr = item(depth + 1);
        return v;
      }
      case VECSXP: case EXPRSXP: {
        auto v = std::make_shared<Node>();
        v->type = type;
        const int64_t len = vec_length();
        check_count(len, 4);
        v->items.reserve((size_t)len);
        for (int64_t i = 0; i < len; ++i) v->items.push_back(item(depth + 1));
        if (has_attr) v->attr = item(depth + 1);
        return v;
      }
      case S4SXP: {
        auto v = std::make_shared<Node>();
        v->type = S4SXP;
        if (has_attr) v->attr = item(depth + 1);
        return v;
      }
      case ALTREP_SXP: {
        // info = pairlist(class sym, package sym, type); state; attributes.  The compact
        // integer / real sequences are expanded; other classes keep their serialized state
        // when it is a plain vector (e.g. wrapper / deferred-string states).
        NodeP info = item(depth + 1);
        NodeP state = item(depth + 1);
        NodeP attr = item(depth + 1);
        std::string cls;
        if (info && !info->items.empty() && info->items[0] && !info->items[0]->strs.empty())
          cls = info->items[0]->strs[0];
        auto v = std::make_shared<Node>();
        if ((cls == "compact_intseq" || cls == "compact_realseq") && state &&
            state->type == REALSXP && state->real.size() == 3) {
          const double len = state->real[0], start = state->real[1], inc = state->real[2];
          if (!(len >= 0 && len <= 4e9)) throw ParseError{"bad compact sequence"};
          const int64_t L = (int64_t)len;
          if (cls == "compact_intseq") {
            v->type = INTSXP;
            v->ints.resize((size_t)L);
            for (int64_t i = 0; i < L; ++i) v->ints[(size_t)i] = (int32_t)(start + inc * (double)i);
          } else {
            v->type = REALSXP;
            v->real.resize((size_t)L);
            for (int64_t i = 0; i < L; ++i) v->real[(size_t)i] = start + inc * (double)i;
          }
        } else if (state && (state->type == VECSXP || state->type == REALSXP ||
                             state->type == INTSXP || state->type == STRSXP)) {
          *v = *(state->type == VECSXP && !state->items.empty() ? state->items[0] : state);
        } else {
          throw ParseError{"unsupported ALTREP class '" + cls + "'"};
        }
        if (attr && attr->type == LISTSXP) v->attr = attr;
        return v;
      }
      default:
        throw ParseError{"unsupported R object type " + std::to_string(type)};
    }
  }
};

thread_local std::string g_rds_err;

int rds_fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_rds_err = buf;
  return code;
}

}  // namespace

struct dcor_rds {
  NodeP root;                       // the data.frame (VECSXP with names)
  std::vector<std::string> names;
  int64_t nrow = 0;
};

namespace {

const Node* column(const dcor_rds* h, const char* name) {
  for (size_t j = 0; j < h->names.size(); ++j)
    if (h->names[j] == name) return h->root->items[j].get();
  return nullptr;
}

}  // namespace

extern "C" {

const char* dcor_rds_last_error(void) { return g_rds_err.c_str(); }

int dcor_rds_open(const char* path, dcor_rds** out) {
  if (!path || !out) return rds_fail(DCOR_EINVAL, "rds_open: null argument");
  *out = nullptr;
  gzFile f = gzopen(path, "rb");  // reads gzip and plain files alike
  if (!f) return rds_fail(DCOR_EINVAL, "rds_open: cannot open %s", path);
  std::vector<unsigned char> buf;
  unsigned char chunk[1 << 16];
  for (;;) {
    const int r = gzread(f, chunk, sizeof(chunk));
    if (r < 0) {
      gzclose(f);
      return rds_fail(DCOR_EINVAL, "rds_open: %s: decompression error", path);
    }
    if (r == 0) break;
    if (buf.size() + (size_t)r > ((size_t)8 << 30)) {
      gzclose(f);
      return rds_fail(DCOR_ENOMEM, "rds_open: %s: larger than 8 GiB uncompressed", path);
    }
    buf.insert(buf.end(), chunk, chunk + r);
  }
  gzclose(f);
  std::unique_ptr<dcor_rds> h(new dcor_rds());
  try {
    h->root = Reader(buf.data(), buf.size()).parse();
  } catch (const ParseError& e) {
    return rds_fail(DCOR_EINVAL, "rds_open: %s: %s", path, e.msg.c_str());
  } catch (const std::bad_alloc&) {
    return rds_fail(DCOR_ENOMEM, "rds_open: %s: out of memory", path);
  }
  const Node& r = *h->root;
  if (r.type != VECSXP) return rds_fail(DCOR_EINVAL, "rds_open: %s: not a list / data.frame", path);
  NodeP nm = r.get_attr("names");
  if (!nm || nm->type != STRSXP || nm->strs.size() != r.items.size())
    return rds_fail(DCOR_EINVAL, "rds_open: %s: list without names", path);
  h->names = nm->strs;
  h->nrow = r.items.empty() ? 0 : r.items[0]->length();
  for (const NodeP& c : r.items)
    if (c->length() != h->nrow)
      return rds_fail(DCOR_EINVAL, "rds_open: %s: columns of unequal length", path);
  *out = h.release();
  return DCOR_OK;
}

void dcor_rds_close(dcor_rds* h) { delete h; }

int64_t dcor_rds_ncol(const dcor_rds* h) { return h ? (int64_t)h->names.size() : -1; }
int64_t dcor_rds_nrow(const dcor_rds* h) { return h ? h->nrow : -1; }

int dcor_rds_colname(const dcor_rds* h, int64_t j, char* buf, size_t len) {
  if (!h || j < 0 || j >= (int64_t)h->names.size() || !buf || len == 0)
    return rds_fail(DCOR_EINVAL, "rds_colname: bad arguments");
  std::snprintf(buf, len, "%s", h->names[(size_t)j].c_str());
  return DCOR_OK;
}

int dcor_rds_coltype(const dcor_rds* h, const char* name) {
  if (!h || !name) return -1;
  const Node* c = column(h, name);
  return c ? c->type : -1;
}

int dcor_rds_real(const dcor_rds* h, const char* name, double* out) {
  if (!h || !name || !out) return rds_fail(DCOR_EINVAL, "rds_real: null argument");
  const Node* c = column(h, name);
  if (!c) return rds_fail(DCOR_EINVAL, "rds_real: no column '%s'", name);
  if (c->type == REALSXP) {
    std::memcpy(out, c->real.data(), sizeof(double) * c->real.size());
  } else if (c->type == INTSXP || c->type == LGLSXP) {  // as.numeric: NA_integer_ -> NA_real_
    for (size_t i = 0; i < c->ints.size(); ++i)
      out[i] = c->ints[i] == R_NA_INT ? NAN : (double)c->ints[i];
  } else {
    return rds_fail(DCOR_EINVAL, "rds_real: column '%s' is not numeric (type %d)", name, c->type);
  }
  return DCOR_OK;
}

// out[i] = (column[i] == value): strings compare by text (NA -> 0); factors by level label;
// numeric columns by value == strtod(value) (R's `%in%` coerces to character, so "2" matches 2).
int dcor_rds_eq(const dcor_rds* h, const char* name, const char* value, uint8_t* out) {
  if (!h || !name || !value || !out) return rds_fail(DCOR_EINVAL, "rds_eq: null argument");
  const Node* c = column(h, name);
  if (!c) return rds_fail(DCOR_EINVAL, "rds_eq: no column '%s'", name);
  if (c->type == STRSXP) {
    for (size_t i = 0; i < c->strs.size(); ++i) out[i] = !c->str_na[i] && c->strs[i] == value;
    return DCOR_OK;
  }
  NodeP lev = c->get_attr("levels");
  if (c->type == INTSXP && lev && lev->type == STRSXP) {
    for (size_t i = 0; i < c->ints.size(); ++i) {
      const int32_t k = c->ints[i];
      out[i] = k != R_NA_INT && k >= 1 && (size_t)k <= lev->strs.size() && lev->strs[(size_t)k - 1] == value;
    }
    return DCOR_OK;
  }
  char* end = nullptr;
  const double v = std::strtod(value, &end);
  if (end == value) {
    std::memset(out, 0, (size_t)h->nrow);
    return DCOR_OK;
  }
  if (c->type == REALSXP) {
    for (size_t i = 0; i < c->real.size(); ++i) out[i] = c->real[i] == v;
  } else if (c->type == INTSXP || c->type == LGLSXP) {
    for (size_t i = 0; i < c->ints.size(); ++i) out[i] = c->ints[i] != R_NA_INT && (double)c->ints[i] == v;
  } else {
    return rds_fail(DCOR_EINVAL, "rds_eq: column '%s' has type %d", name, c->type);
  }
  return DCOR_OK;
}

int dcor_hrs_wave(const char* path, const char* wave, double* age, double* bmi, int64_t cap,
                  int64_t* n) {
  if (!path || !wave || !n) return rds_fail(DCOR_EINVAL, "hrs_wave: null argument");
  dcor_rds* h = nullptr;
  if (int st = dcor_rds_open(path, &h)) return st;
  std::unique_ptr<dcor_rds, void (*)(dcor_rds*)> guard(h, dcor_rds_close);
  const int64_t N = h->nrow;
  std::vector<uint8_t> keep((size_t)N);
  std::vector<double> a((size_t)N), b((size_t)N);
  if (int st = dcor_rds_eq(h, "wave", wave, keep.data())) return st;   // filter(wave %in% ..)
  if (int st = dcor_rds_real(h, "agey_e", a.data())) return st;         // transmute(age = agey_e,
  if (int st = dcor_rds_real(h, "bmi", b.data())) return st;            //           bmi)
  int64_t m = 0;
  for (int64_t i = 0; i < N; ++i) {
    if (!keep[(size_t)i] || std::isnan(a[(size_t)i]) || std::isnan(b[(size_t)i])) continue;  // drop_na
    if (m < cap && age && bmi) { age[m] = a[(size_t)i]; bmi[m] = b[(size_t)i]; }
    ++m;
  }
  *n = m;
  if (m > cap && (age || bmi))
    return rds_fail(DCOR_EINVAL, "hrs_wave: %lld rows, capacity %lld", (long long)m, (long long)cap);
  return DCOR_OK;
}

}  // extern "C"
