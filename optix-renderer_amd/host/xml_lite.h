// Minimal XML DOM reader for Nori scene files: elements, attributes, comments and
// the XML declaration. Nori scenes carry no text content that matters, so
// character data is skipped. Replaces the reference's use of pugixml inside
// loadFromXML (src/utils/parser.cpp:28-35).
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace nh {

struct XmlNode {
    std::string name;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XmlNode>> children;
    size_t offset = 0;  // byte offset of '<' in the source, for error messages

    const std::string *attr(const std::string &key) const {
        for (auto &kv : attrs)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
};

struct XmlError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// Parse a whole document; returns the root element.
std::unique_ptr<XmlNode> xml_parse(const std::string &text);
// Convert a byte offset to "row R, col C" like the reference's error helper.
std::string xml_position(const std::string &text, size_t offset);

}  // namespace nh
