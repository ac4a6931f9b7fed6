// Minimal JSON value / parser / serializer for the operator core.
//
// Kubernetes objects cross the Python<->C++ boundary as JSON text.  Objects
// keep insertion order (so a pod template round-trips unchanged) and the
// serializer can emit Go `encoding/json`-compatible bytes: struct fields in
// declaration order, map keys sorted, HTML-sensitive characters escaped as
// < > & -- which is what makes TF_CONFIG byte-identical to
// the reference (pkg/controller.v1/tensorflow/pod_test.go:230-281).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace toa {

class Json {
 public:
  enum class Type { Null, Bool, Int, Double, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::vector<std::pair<std::string, Json>>;

  Json() : type_(Type::Null) {}
  Json(std::nullptr_t) : type_(Type::Null) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(int v) : type_(Type::Int), i_(v) {}
  Json(int64_t v) : type_(Type::Int), i_(v) {}
  Json(double v) : type_(Type::Double), d_(v) {}
  Json(const char* s) : type_(Type::String), s_(s) {}
  Json(std::string s) : type_(Type::String), s_(std::move(s)) {}
  Json(Array a) : type_(Type::Array), a_(std::make_shared<Array>(std::move(a))) {}
  Json(Object o) : type_(Type::Object), o_(std::make_shared<Object>(std::move(o))) {}

  static Json object() { return Json(Object{}); }
  static Json array() { return Json(Array{}); }
  static Json parse(const std::string& text);

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_number() const { return type_ == Type::Int || type_ == Type::Double; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool(bool dflt = false) const { return type_ == Type::Bool ? b_ : dflt; }
  int64_t as_int(int64_t dflt = 0) const {
    if (type_ == Type::Int) return i_;
    if (type_ == Type::Double) return (int64_t)d_;
    return dflt;
  }
  double as_double(double dflt = 0) const {
    if (type_ == Type::Double) return d_;
    if (type_ == Type::Int) return (double)i_;
    return dflt;
  }
  const std::string& as_string() const {
    static const std::string empty;
    return type_ == Type::String ? s_ : empty;
  }
  std::string str(const std::string& dflt = "") const { return type_ == Type::String ? s_ : dflt; }

  // array access
  size_t size() const {
    if (type_ == Type::Array) return a_->size();
    if (type_ == Type::Object) return o_->size();
    return 0;
  }
  const Json& operator[](size_t i) const { return (*a_)[i]; }
  Json& at(size_t i) {
    detach();
    return (*a_)[i];
  }
  void push_back(Json v) {
    if (type_ == Type::Null) *this = array();
    detach();
    a_->push_back(std::move(v));
  }
  const Array& items() const {
    static const Array empty;
    return type_ == Type::Array ? *a_ : empty;
  }
  Array& mutable_items() {
    if (type_ == Type::Null) *this = array();
    detach();
    return *a_;
  }

  // object access
  bool has(const std::string& k) const { return find(k) != nullptr; }
  const Json* find(const std::string& k) const;
  const Json& get(const std::string& k) const;  // Null if absent
  Json& operator[](const std::string& k);        // insert Null if absent (object)
  void set(const std::string& k, Json v) { (*this)[k] = std::move(v); }
  bool erase(const std::string& k);
  const Object& fields() const {
    static const Object empty;
    return type_ == Type::Object ? *o_ : empty;
  }
  Object& mutable_fields() {
    if (type_ == Type::Null) *this = object();
    detach();
    return *o_;
  }
  // Path helper: get("a").get("b") without creating.
  const Json& path(std::initializer_list<const char*> keys) const;

  std::string dump(bool sort_keys = false) const;
  bool operator==(const Json& o) const;
  bool operator!=(const Json& o) const { return !(*this == o); }

 private:
  void detach();  // copy-on-write for shared containers
  void dump_to(std::string& out, bool sort_keys) const;

  Type type_;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
};

std::string json_escape(const std::string& s);

}  // namespace toa
