#include "json.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace gsdr_rt {

class JsonParser {
 public:
  explicit JsonParser(const char* s) : p(s) {}

  bool parseDocument(Json& out, std::string& err) {
    if (!value(out, err, 0)) return false;
    ws();
    if (*p != '\0') {
      err = "trailing characters";
      return false;
    }
    return true;
  }

 private:
  const char* p;

  void ws() {
    while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') ++p;
  }

  bool literal(const char* lit) {
    const size_t n = strlen(lit);
    if (strncmp(p, lit, n) != 0) return false;
    p += n;
    return true;
  }

  static void appendUtf8(std::string& s, unsigned cp) {
    if (cp < 0x80) {
      s += (char)cp;
    } else if (cp < 0x800) {
      s += (char)(0xC0 | (cp >> 6));
      s += (char)(0x80 | (cp & 0x3F));
    } else {
      s += (char)(0xE0 | (cp >> 12));
      s += (char)(0x80 | ((cp >> 6) & 0x3F));
      s += (char)(0x80 | (cp & 0x3F));
    }
  }

  bool str(std::string& out, std::string& err) {
    if (*p != '"') {
      err = "expected string";
      return false;
    }
    ++p;
    while (*p != '"') {
      if (*p == '\0') {
        err = "unterminated string";
        return false;
      }
      if (*p == '\\') {
        ++p;
        switch (*p) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            unsigned cp = 0;
            for (int i = 1; i <= 4; ++i) {
              const char c = p[i];
              cp <<= 4;
              if (c >= '0' && c <= '9') cp |= c - '0';
              else if (c >= 'a' && c <= 'f') cp |= c - 'a' + 10;
              else if (c >= 'A' && c <= 'F') cp |= c - 'A' + 10;
              else {
                err = "bad \\u escape";
                return false;
              }
            }
            appendUtf8(out, cp);
            p += 4;
            break;
          }
          default: err = "bad escape"; return false;
        }
        ++p;
      } else {
        out += *p++;
      }
    }
    ++p;
    return true;
  }

  bool value(Json& v, std::string& err, int depth) {
    if (depth > 64) {
      err = "nesting too deep";
      return false;
    }
    ws();
    if (*p == '{') {
      ++p;
      v.mType = Json::Type::Object;
      ws();
      if (*p == '}') {
        ++p;
        return true;
      }
      for (;;) {
        ws();
        std::string key;
        if (!str(key, err)) return false;
        ws();
        if (*p != ':') {
          err = "expected ':'";
          return false;
        }
        ++p;
        Json child;
        if (!value(child, err, depth + 1)) return false;
        v.mObject[key] = std::move(child);
        ws();
        if (*p == ',') {
          ++p;
          continue;
        }
        if (*p == '}') {
          ++p;
          return true;
        }
        err = "expected ',' or '}'";
        return false;
      }
    }
    if (*p == '[') {
      ++p;
      v.mType = Json::Type::Array;
      ws();
      if (*p == ']') {
        ++p;
        return true;
      }
      for (;;) {
        Json child;
        if (!value(child, err, depth + 1)) return false;
        v.mArray.push_back(std::move(child));
        ws();
        if (*p == ',') {
          ++p;
          continue;
        }
        if (*p == ']') {
          ++p;
          return true;
        }
        err = "expected ',' or ']'";
        return false;
      }
    }
    if (*p == '"') {
      v.mType = Json::Type::String;
      return str(v.mString, err);
    }
    if (literal("true")) {
      v.mType = Json::Type::Bool;
      v.mBool = true;
      return true;
    }
    if (literal("false")) {
      v.mType = Json::Type::Bool;
      v.mBool = false;
      return true;
    }
    if (literal("null")) {
      v.mType = Json::Type::Null;
      return true;
    }
    char* end = nullptr;
    const double d = strtod(p, &end);
    if (end == p) {
      err = "unexpected character";
      return false;
    }
    v.mType = Json::Type::Number;
    v.mNumber = d;
    p = end;
    return true;
  }
};

namespace {
void dumpString(const std::string& s, std::string& out) {
  out += '"';
  for (const char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof(buf), "\\u%04x", (unsigned)(unsigned char)c);
          out += buf;
        } else {
          out += c;
        }
    }
  }
  out += '"';
}

void dumpValue(const Json& v, std::string& out) {
  switch (v.type()) {
    case Json::Type::Null: out += "null"; break;
    case Json::Type::Bool: out += v.boolean() ? "true" : "false"; break;
    case Json::Type::Number: {
      char buf[40];
      snprintf(buf, sizeof(buf), "%.17g", v.number());
      out += buf;
      break;
    }
    case Json::Type::String: dumpString(v.string(), out); break;
    case Json::Type::Array: {
      out += '[';
      bool first = true;
      for (const Json& e : v.array()) {
        if (!first) out += ',';
        first = false;
        dumpValue(e, out);
      }
      out += ']';
      break;
    }
    case Json::Type::Object: {
      out += '{';
      bool first = true;
      for (const auto& kv : v.object()) {
        if (!first) out += ',';
        first = false;
        dumpString(kv.first, out);
        out += ':';
        dumpValue(kv.second, out);
      }
      out += '}';
      break;
    }
  }
}
}  // namespace

std::string Json::dump() const {
  std::string out;
  dumpValue(*this, out);
  return out;
}

bool Json::parse(const char* text, Json& out, std::string& error) {
  out = Json();
  if (text == nullptr) {
    error = "null JSON text";
    return false;
  }
  JsonParser parser(text);
  return parser.parseDocument(out, error);
}

}  // namespace gsdr_rt
