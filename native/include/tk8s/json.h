// Minimal JSON writer shared by every tk8s native component. No HIP dependency: the AMD SMI
// health tool and the CPU-only pieces include it without pulling in the HIP runtime.
#pragma once

#include <cstdint>
#include <cstdio>
#include <sstream>
#include <string>
#include <vector>

namespace tk8s {

// Minimal JSON object writer: enough for flat records and arrays of records.
class Json {
 public:
  Json& kv(const std::string& k, const std::string& v) { key(k); str(v); return *this; }
  Json& kv(const std::string& k, const char* v) { return kv(k, std::string(v)); }
  Json& kv(const std::string& k, double v) { key(k); num(v); return *this; }
  Json& kv(const std::string& k, int64_t v) { key(k); os_ << v; return *this; }
  Json& kv(const std::string& k, uint64_t v) { key(k); os_ << v; return *this; }
  Json& kv(const std::string& k, int v) { return kv(k, static_cast<int64_t>(v)); }
  Json& kv(const std::string& k, unsigned v) { return kv(k, static_cast<uint64_t>(v)); }
  Json& kv(const std::string& k, bool v) { key(k); os_ << (v ? "true" : "false"); return *this; }
  Json& raw(const std::string& k, const std::string& json) { key(k); os_ << json; return *this; }
  std::string str() const { return "{" + os_.str() + "}"; }

  static std::string escape(const std::string& s) {
    std::string o = "\"";
    for (char c : s) {
      switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\t': o += "\\t"; break;
        default:
          if (static_cast<unsigned char>(c) < 0x20) {
            char buf[8];
            std::snprintf(buf, sizeof buf, "\\u%04x", c);
            o += buf;
          } else {
            o += c;
          }
      }
    }
    return o + "\"";
  }
  static std::string array(const std::vector<std::string>& items) {
    std::string o = "[";
    for (size_t i = 0; i < items.size(); ++i) o += (i ? "," : "") + items[i];
    return o + "]";
  }

 private:
  void key(const std::string& k) {
    if (!first_) os_ << ",";
    first_ = false;
    os_ << escape(k) << ":";
  }
  void str(const std::string& v) { os_ << escape(v); }
  void num(double v) {
    char buf[64];
    // 9 significant digits, except for large magnitudes (wall-clock timestamps in ms, ~1.8e12):
    // those keep three decimals, or "%.9g" would round them to whole seconds
    if (v >= 1e6 || v <= -1e6) std::snprintf(buf, sizeof buf, "%.3f", v);
    else std::snprintf(buf, sizeof buf, "%.9g", v);
    os_ << buf;
  }
  std::ostringstream os_;
  bool first_ = true;
};

}  // namespace tk8s
