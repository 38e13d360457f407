// Minimal JSON reader for node / queue parameters (the reference uses nlohmann::json, which is
// fetched from the network at configure time and is not available here). Objects, arrays,
// strings (with \" \\ \/ \b \f \n \r \t \uXXXX escapes), numbers, booleans and null.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

namespace gsdr_rt {

class Json {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };

  static bool parse(const char* text, Json& out, std::string& error);
  // Compact JSON text of this value (numbers with 17 significant digits: they parse back exactly).
  std::string dump() const;

  Type type() const { return mType; }
  bool isNull() const { return mType == Type::Null; }
  bool isNumber() const { return mType == Type::Number; }
  bool isString() const { return mType == Type::String; }
  bool isArray() const { return mType == Type::Array; }
  bool isObject() const { return mType == Type::Object; }
  bool isBool() const { return mType == Type::Bool; }

  double number() const { return mNumber; }
  bool boolean() const { return mBool; }
  const std::string& string() const { return mString; }
  const std::vector<Json>& array() const { return mArray; }
  const std::map<std::string, Json>& object() const { return mObject; }

  bool contains(const std::string& key) const { return mType == Type::Object && mObject.count(key) != 0; }
  const Json* get(const std::string& key) const {
    if (mType != Type::Object) return nullptr;
    auto it = mObject.find(key);
    return it == mObject.end() ? nullptr : &it->second;
  }

 private:
  friend class JsonParser;
  Type mType = Type::Null;
  bool mBool = false;
  double mNumber = 0.0;
  std::string mString;
  std::vector<Json> mArray;
  std::map<std::string, Json> mObject;
};

}  // namespace gsdr_rt
