#include "json.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cerrno>

namespace toa {

void Json::detach() {
  if (type_ == Type::Array && a_ && a_.use_count() > 1) a_ = std::make_shared<Array>(*a_);
  if (type_ == Type::Object && o_ && o_.use_count() > 1) o_ = std::make_shared<Object>(*o_);
}

const Json* Json::find(const std::string& k) const {
  if (type_ != Type::Object) return nullptr;
  for (const auto& kv : *o_)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

const Json& Json::get(const std::string& k) const {
  static const Json null;
  const Json* p = find(k);
  return p ? *p : null;
}

const Json& Json::path(std::initializer_list<const char*> keys) const {
  const Json* cur = this;
  for (const char* k : keys) {
    cur = &cur->get(k);
    if (cur->is_null()) return *cur;
  }
  return *cur;
}

Json& Json::operator[](const std::string& k) {
  if (type_ == Type::Null) *this = object();
  if (type_ != Type::Object) throw std::runtime_error("json: not an object (key " + k + ")");
  detach();
  for (auto& kv : *o_)
    if (kv.first == k) return kv.second;
  o_->emplace_back(k, Json());
  return o_->back().second;
}

bool Json::erase(const std::string& k) {
  if (type_ != Type::Object) return false;
  detach();
  auto it = std::find_if(o_->begin(), o_->end(), [&](const auto& kv) { return kv.first == k; });
  if (it == o_->end()) return false;
  o_->erase(it);
  return true;
}

bool Json::operator==(const Json& o) const {
  if (is_number() && o.is_number()) {
    if (type_ == Type::Int && o.type_ == Type::Int) return i_ == o.i_;
    return as_double() == o.as_double();
  }
  if (type_ != o.type_) return false;
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::String: return s_ == o.s_;
    case Type::Array: return *a_ == *o.a_;
    case Type::Object: {
      // order-insensitive object equality
      if (o_->size() != o.o_->size()) return false;
      for (const auto& kv : *o_) {
        const Json* v = o.find(kv.first);
        if (!v || !(*v == kv.second)) return false;
      }
      return true;
    }
    default: return false;
  }
}

// ---------------------------------------------------------------------------
// serializer (Go-compatible escaping)
// ---------------------------------------------------------------------------
std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '<': out += "\\u003c"; break;
      case '>': out += "\\u003e"; break;
      case '&': out += "\\u0026"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  return out;
}

static void dump_double(std::string& out, double d) {
  if (std::isfinite(d) && d == std::floor(d) && std::fabs(d) < 1e15) {
    char buf[32];
    snprintf(buf, sizeof buf, "%lld", (long long)d);
    out += buf;
    return;
  }
  char buf[40];
  snprintf(buf, sizeof buf, "%.17g", d);
  // shortest round-trip representation
  for (int p = 1; p <= 17; ++p) {
    char b2[40];
    snprintf(b2, sizeof b2, "%.*g", p, d);
    if (std::strtod(b2, nullptr) == d) {
      out += b2;
      return;
    }
  }
  out += buf;
}

void Json::dump_to(std::string& out, bool sort_keys) const {
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Int: out += std::to_string(i_); break;
    case Type::Double: dump_double(out, d_); break;
    case Type::String:
      out += '"';
      out += json_escape(s_);
      out += '"';
      break;
    case Type::Array: {
      out += '[';
      bool first = true;
      for (const auto& v : *a_) {
        if (!first) out += ',';
        first = false;
        v.dump_to(out, sort_keys);
      }
      out += ']';
      break;
    }
    case Type::Object: {
      out += '{';
      std::vector<const std::pair<std::string, Json>*> kvs;
      for (const auto& kv : *o_) kvs.push_back(&kv);
      if (sort_keys)
        std::sort(kvs.begin(), kvs.end(), [](auto* a, auto* b) { return a->first < b->first; });
      bool first = true;
      for (auto* kv : kvs) {
        if (!first) out += ',';
        first = false;
        out += '"';
        out += json_escape(kv->first);
        out += "\":";
        kv->second.dump_to(out, sort_keys);
      }
      out += '}';
      break;
    }
  }
}

std::string Json::dump(bool sort_keys) const {
  std::string out;
  dump_to(out, sort_keys);
  return out;
}

// ---------------------------------------------------------------------------
// parser
// ---------------------------------------------------------------------------
namespace {
struct Parser {
  const std::string& s;
  size_t i = 0;
  explicit Parser(const std::string& t) : s(t) {}

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json parse error: ") + what + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\t' || s[i] == '\r')) ++i;
  }
  bool eat(char c) {
    ws();
    if (i < s.size() && s[i] == c) {
      ++i;
      return true;
    }
    return false;
  }
  void expect(char c) {
    if (!eat(c)) fail("unexpected character");
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i + 4 > s.size()) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    ws();
    if (i >= s.size() || s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (true) {
      if (i >= s.size()) fail("unterminated string");
      char c = s[i++];
      if (c == '"') break;
      if (c == '\\') {
        if (i >= s.size()) fail("bad escape");
        char e = s[i++];
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00 && i + 1 < s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              i += 2;
              uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            utf8(out, cp);
            break;
          }
          default: fail("bad escape");
        }
      } else {
        out += c;
      }
    }
    return out;
  }
  Json value(int depth = 0) {
    if (depth > 512) fail("nesting too deep");
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      ++i;
      Json o = Json::object();
      auto& f = o.mutable_fields();
      if (eat('}')) return o;
      while (true) {
        std::string k = str();
        expect(':');
        Json v = value(depth + 1);
        bool replaced = false;
        for (auto& kv : f)
          if (kv.first == k) {
            kv.second = std::move(v);
            replaced = true;
            break;
          }
        if (!replaced) f.emplace_back(std::move(k), std::move(v));
        if (eat(',')) continue;
        expect('}');
        return o;
      }
    }
    if (c == '[') {
      ++i;
      Json a = Json::array();
      auto& it = a.mutable_items();
      if (eat(']')) return a;
      while (true) {
        it.push_back(value(depth + 1));
        if (eat(',')) continue;
        expect(']');
        return a;
      }
    }
    if (c == '"') return Json(str());
    if (s.compare(i, 4, "true") == 0) { i += 4; return Json(true); }
    if (s.compare(i, 5, "false") == 0) { i += 5; return Json(false); }
    if (s.compare(i, 4, "null") == 0) { i += 4; return Json(); }
    // number
    size_t st = i;
    bool is_float = false;
    if (s[i] == '-') ++i;
    while (i < s.size() && ((s[i] >= '0' && s[i] <= '9') || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                            s[i] == '+' || s[i] == '-')) {
      if (s[i] == '.' || s[i] == 'e' || s[i] == 'E') is_float = true;
      ++i;
    }
    if (st == i) fail("unexpected token");
    std::string num = s.substr(st, i - st);
    if (!is_float) {
      errno = 0;
      long long v = std::strtoll(num.c_str(), nullptr, 10);
      if (errno == 0) return Json((int64_t)v);
    }
    return Json(std::strtod(num.c_str(), nullptr));
  }
};
}  // namespace

Json Json::parse(const std::string& text) {
  Parser p(text);
  Json v = p.value();
  p.ws();
  if (p.i != text.size()) p.fail("trailing characters");
  return v;
}

}  // namespace toa
