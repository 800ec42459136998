#include "xml_lite.h"

#include <cctype>
#include <cstring>

namespace nh {

namespace {

struct Parser {
    const std::string &s;
    size_t i = 0;
    explicit Parser(const std::string &src) : s(src) {}

    [[noreturn]] void fail(const std::string &msg) const {
        throw XmlError(msg + " (at " + xml_position(s, i) + ")");
    }
    bool starts(const char *lit) const { return s.compare(i, std::strlen(lit), lit) == 0; }
    void skip_ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
    }
    void skip_misc() {
        // whitespace, comments, declarations, processing instructions, DOCTYPE
        for (;;) {
            skip_ws();
            if (starts("<!--")) {
                size_t e = s.find("-->", i + 4);
                if (e == std::string::npos) fail("unterminated comment");
                i = e + 3;
            } else if (starts("<?")) {
                size_t e = s.find("?>", i + 2);
                if (e == std::string::npos) fail("unterminated declaration");
                i = e + 2;
            } else if (starts("<!")) {
                size_t e = s.find('>', i + 2);
                if (e == std::string::npos) fail("unterminated markup");
                i = e + 1;
            } else {
                return;
            }
        }
    }
    std::string name() {
        size_t b = i;
        while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == ':' || s[i] == '.'))
            ++i;
        if (b == i) fail("expected a name");
        return s.substr(b, i - b);
    }
    static std::string unescape(const std::string &v) {
        std::string out;
        out.reserve(v.size());
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] != '&') { out.push_back(v[k]); continue; }
            size_t e = v.find(';', k);
            if (e == std::string::npos) { out.push_back('&'); continue; }
            std::string ent = v.substr(k + 1, e - k - 1);
            if (ent == "amp") out.push_back('&');
            else if (ent == "lt") out.push_back('<');
            else if (ent == "gt") out.push_back('>');
            else if (ent == "quot") out.push_back('"');
            else if (ent == "apos") out.push_back('\'');
            else { out.append(v, k, e - k + 1); }
            k = e;
        }
        return out;
    }
    std::unique_ptr<XmlNode> element() {
        if (i >= s.size() || s[i] != '<') fail("expected '<'");
        auto node = std::make_unique<XmlNode>();
        node->offset = i;
        ++i;
        node->name = name();
        for (;;) {
            skip_ws();
            if (i >= s.size()) fail("unexpected end of file in tag");
            if (starts("/>")) { i += 2; return node; }
            if (s[i] == '>') { ++i; break; }
            std::string key = name();
            skip_ws();
            if (i >= s.size() || s[i] != '=') fail("expected '=' after attribute name");
            ++i;
            skip_ws();
            if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) fail("expected quoted attribute value");
            char q = s[i++];
            size_t e = s.find(q, i);
            if (e == std::string::npos) fail("unterminated attribute value");
            node->attrs.emplace_back(key, unescape(s.substr(i, e - i)));
            i = e + 1;
        }
        // content
        for (;;) {
            // character data is ignored (Nori scenes have none that matters)
            while (i < s.size() && s[i] != '<') ++i;
            if (i >= s.size()) fail("unterminated element <" + node->name + ">");
            if (starts("</")) {
                i += 2;
                std::string closing = name();
                if (closing != node->name) fail("mismatched closing tag </" + closing + "> for <" + node->name + ">");
                skip_ws();
                if (i >= s.size() || s[i] != '>') fail("expected '>'");
                ++i;
                return node;
            }
            if (starts("<!--") || starts("<?") || starts("<!")) {
                skip_misc();
                continue;
            }
            node->children.push_back(element());
        }
    }
};

}  // namespace

std::string xml_position(const std::string &text, size_t offset) {
    int line = 1;
    size_t linestart = 0;
    for (size_t k = 0; k < offset && k < text.size(); ++k)
        if (text[k] == '\n') { ++line; linestart = k + 1; }
    return "row " + std::to_string(line) + ", col " + std::to_string(offset - linestart + 1);
}

std::unique_ptr<XmlNode> xml_parse(const std::string &text) {
    Parser p(text);
    p.skip_misc();
    auto root = p.element();
    p.skip_misc();
    if (p.i != text.size()) p.fail("trailing content after the root element");
    return root;
}

}  // namespace nh
