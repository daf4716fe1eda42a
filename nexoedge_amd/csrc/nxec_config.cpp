// Storage-class and proxy INI files for hosts that drive the coding path
// without the reference's Config singleton (SURVEY §5 "Config / flags": a
// tiny INI reader for the config-1 sample files).
//
// The reference reads these through boost::property_tree's INI parser
// (Config, src/common/config.cc:267-282 classes and the `default = 1` class,
// :664-690 coding / n / k / f / max_chunk_size, :320 misc.repair_using_car)
// and its Config::readIntWithBounds clamping (:692-697).  Here: `[section]`
// headers, `key = value` lines, `;` / `#` comment lines, whitespace trimmed;
// a repeated section or key, a key outside any section or a line that is
// none of these is a parse error (boost rejects the same).  Values are parsed
// like property_tree's get<int> / get<bool> (integers; 0/1/true/false).
#include <cctype>
#include <cerrno>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>

#include "nxec.h"
#include "nxec_internal.h"

using nxec::set_error;

namespace {

struct Ini {
  std::vector<std::string> order;  // sections in file order
  std::map<std::string, std::map<std::string, std::string>> sec;
};

std::string trim(const std::string &s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) b++;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) e--;
  return s.substr(b, e - b);
}

int read_ini(const char *path, Ini &ini) {
  if (!path) return set_error(NXEC_ERR_INVALID, "ini: null path");
  std::ifstream f(path);
  if (!f) return set_error(NXEC_ERR_INVALID, "ini: cannot open %s", path);
  std::string line, cur;
  bool in_section = false;
  for (int ln = 1; std::getline(f, line); ln++) {
    const std::string t = trim(line);
    if (t.empty() || t[0] == ';' || t[0] == '#') continue;
    if (t[0] == '[') {
      if (t.back() != ']' || t.size() < 3) return set_error(NXEC_ERR_INVALID, "ini %s:%d: bad section header", path, ln);
      cur = trim(t.substr(1, t.size() - 2));
      if (ini.sec.count(cur)) return set_error(NXEC_ERR_INVALID, "ini %s:%d: duplicate section [%s]", path, ln, cur.c_str());
      ini.sec[cur];
      ini.order.push_back(cur);
      in_section = true;
      continue;
    }
    const size_t eq = t.find('=');
    if (eq == std::string::npos || !in_section) return set_error(NXEC_ERR_INVALID, "ini %s:%d: expected key = value", path, ln);
    const std::string key = trim(t.substr(0, eq)), val = trim(t.substr(eq + 1));
    if (key.empty()) return set_error(NXEC_ERR_INVALID, "ini %s:%d: empty key", path, ln);
    auto &kv = ini.sec[cur];
    if (kv.count(key)) return set_error(NXEC_ERR_INVALID, "ini %s:%d: duplicate key %s", path, ln, key.c_str());
    kv[key] = val;
  }
  return NXEC_OK;
}

// property_tree get<int>: the whole value is one integer that fits an int
// (Config reads every one of these keys as int; an out-of-range value throws
// there and the key falls back to its default)
bool parse_int(const std::string &v, long long &out) {
  if (v.empty()) return false;
  errno = 0;
  char *end = nullptr;
  out = std::strtoll(v.c_str(), &end, 10);
  return errno == 0 && end && *end == '\0' && out >= INT32_MIN && out <= INT32_MAX;
}

// property_tree get<bool>: 0/1 or true/false
bool parse_bool(const std::string &v, bool &out) {
  std::string l;
  for (char c : v) l += static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  if (l == "1" || l == "true") return out = true, true;
  if (l == "0" || l == "false") return out = false, true;
  return false;
}

// Config::readIntWithBoundsAndDefault (config.cc:692-705): absent or
// unparsable -> dv; otherwise <= min -> min, > max -> max
long long bounded(const std::map<std::string, std::string> &kv, const char *key, long long dv, long long min,
                  long long max) {
  auto it = kv.find(key);
  long long v = 0;
  if (it == kv.end() || !parse_int(it->second, v)) return dv;
  return v <= min ? min : (v > max ? max : v);
}

}  // namespace

extern "C" {

int nxec_storage_classes_load(const char *path, nxec_storage_class *out, int max, int *count) {
  if ((!out && max > 0) || max < 0 || !count)
    return set_error(NXEC_ERR_INVALID, "nxec_storage_classes_load: invalid arguments");
  *count = 0;
  Ini ini;
  if (int rc = read_ini(path, ini)) return rc;
  int ndefault = 0;
  for (const std::string &name : ini.order) {
    const auto &kv = ini.sec[name];
    nxec_storage_class c;
    std::memset(&c, 0, sizeof(c));
    if (name.size() >= sizeof(c.name)) return set_error(NXEC_ERR_INVALID, "storage class name too long: %s", name.c_str());
    std::memcpy(c.name, name.c_str(), name.size() + 1);
    // Config::getCodingScheme (config.cc:664-670, parseCodingScheme :1286-1291): case-insensitive "rs"
    auto cod = kv.find("coding");
    std::string lc;
    if (cod != kv.end())
      for (char ch : cod->second) lc += static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
    c.coding = lc == "rs" ? NXEC_CODING_RS : NXEC_CODING_UNKNOWN;
    c.n = static_cast<int>(bounded(kv, "n", -1, 0, INT32_MAX));
    c.k = static_cast<int>(bounded(kv, "k", -1, 0, INT32_MAX));
    c.f = static_cast<int>(bounded(kv, "f", -1, 0, INT32_MAX));
    c.max_chunk_size = bounded(kv, "max_chunk_size", 0, 0, int64_t(1) << 30);
    // `default` is read with readBool (config.cc:274): required and boolean
    bool def = false;
    auto d = kv.find("default");
    if (d == kv.end() || !parse_bool(d->second, def))
      return set_error(NXEC_ERR_INVALID, "storage class [%s]: missing or non-boolean 'default'", name.c_str());
    c.is_default = def ? 1 : 0;
    if (def && ++ndefault > 1) return set_error(NXEC_ERR_INVALID, "only one default storage class is allowed");
    if (*count < max) out[*count] = c;
    ++*count;
  }
  return NXEC_OK;
}

int nxec_proxy_repair_using_car(const char *path, int *car) {
  if (!car) return set_error(NXEC_ERR_INVALID, "nxec_proxy_repair_using_car: null output");
  *car = 0;
  Ini ini;
  if (int rc = read_ini(path, ini)) return rc;
  // config.cc:320 readBool(_proxyPt, "misc.repair_using_car")
  auto s = ini.sec.find("misc");
  if (s == ini.sec.end()) return set_error(NXEC_ERR_INVALID, "%s: no [misc] section", path);
  auto it = s->second.find("repair_using_car");
  bool v = false;
  if (it == s->second.end() || !parse_bool(it->second, v))
    return set_error(NXEC_ERR_INVALID, "%s: misc.repair_using_car missing or not boolean", path);
  *car = v ? 1 : 0;
  return NXEC_OK;
}

}  // extern "C"
