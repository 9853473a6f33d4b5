// Minimal JSON value (ordered objects) with a strict parser and a Go
// encoding/json-compatible serializer (HTML-safe escaping of <, >, & like Go).
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace p2p {

class Json {
 public:
  enum Type { Null, Bool, Number, String, Array, Object };

  Json() : t_(Null) {}
  Json(std::nullptr_t) : t_(Null) {}
  Json(bool b) : t_(Bool), b_(b) {}
  Json(int v) : t_(Number), n_(v), is_int_(true), i_(v) {}
  Json(long v) : t_(Number), n_((double)v), is_int_(true), i_(v) {}
  Json(long long v) : t_(Number), n_((double)v), is_int_(true), i_(v) {}
  Json(unsigned long v) : t_(Number), n_((double)v), is_int_(true), i_((long long)v) {}
  Json(double v) : t_(Number), n_(v) {}
  Json(const char* s) : t_(String), s_(s) {}
  Json(const std::string& s) : t_(String), s_(s) {}
  Json(std::string&& s) : t_(String), s_(std::move(s)) {}

  static Json array() {
    Json j;
    j.t_ = Array;
    return j;
  }
  static Json object() {
    Json j;
    j.t_ = Object;
    return j;
  }
  template <class T>
  static Json array_of(const std::vector<T>& v) {
    Json j = array();
    for (auto& x : v) j.push(Json(x));
    return j;
  }

  Type type() const { return t_; }
  bool is_null() const { return t_ == Null; }
  bool is_string() const { return t_ == String; }
  bool is_object() const { return t_ == Object; }
  bool is_array() const { return t_ == Array; }
  bool is_number() const { return t_ == Number; }
  bool is_bool() const { return t_ == Bool; }

  const std::string& str() const;
  double num() const;
  long long integer() const;
  bool boolean() const;

  // arrays
  void push(Json v);
  size_t size() const;
  const Json& at(size_t i) const;
  const std::vector<Json>& items() const { return arr_; }

  // objects (insertion-ordered)
  Json& set(const std::string& k, Json v);
  bool has(const std::string& k) const;
  const Json& get(const std::string& k) const;  // Null json if absent
  const std::vector<std::pair<std::string, Json>>& fields() const { return obj_; }
  std::string get_string(const std::string& k, const std::string& def = "") const;
  double get_number(const std::string& k, double def) const;
  bool get_bool(const std::string& k, bool def) const;

  std::string dump() const;
  // sorted_keys: Go map[string]any (gin.H) ordering
  std::string dump_sorted() const;

  static Json parse(const std::string& text);  // throws JsonError

 private:
  void dump_to(std::string& out, bool sorted) const;
  Type t_;
  bool b_ = false;
  double n_ = 0;
  bool is_int_ = false;
  long long i_ = 0;
  std::string s_;
  std::vector<Json> arr_;
  std::vector<std::pair<std::string, Json>> obj_;
};

struct JsonError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

std::string json_escape(const std::string& s);

}  // namespace p2p
