// xml_lite.h — minimal XML reader for MJCF scene files (elements + attributes only).
// Handles <?..?>, <!-- -->, <!DOCTYPE>, self-closing tags, quoted attributes and the five
// predefined entities.  Text content is ignored (MJCF carries everything in attributes).
#pragma once
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace sspp {

struct XNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XNode>> kids;
    const std::string* get(const char* name) const {
        for (auto& a : attrs)
            if (a.first == name) return &a.second;
        return nullptr;
    }
};

class XmlReader {
public:
    explicit XmlReader(const std::string& s) : s_(s), i_(0) {}

    std::unique_ptr<XNode> parse() {
        std::unique_ptr<XNode> root;
        while (true) {
            skip_misc();
            if (i_ >= s_.size()) break;
            if (s_[i_] != '<') throw err("expected '<'");
            auto n = element();
            if (!root) root = std::move(n);
        }
        if (!root) throw err("empty document");
        return root;
    }

private:
    const std::string& s_;
    size_t i_;

    std::runtime_error err(const char* what) const {
        size_t line = 1;
        for (size_t k = 0; k < i_ && k < s_.size(); ++k) line += s_[k] == '\n';
        return std::runtime_error(std::string("xml: ") + what + " at line " + std::to_string(line));
    }
    bool starts(const char* p) const { return s_.compare(i_, std::strlen(p), p) == 0; }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
    }
    void skip_to(const char* end) {
        size_t k = s_.find(end, i_);
        if (k == std::string::npos) throw err("unterminated construct");
        i_ = k + std::strlen(end);
    }
    // skip whitespace, text, comments, declarations, processing instructions
    void skip_misc() {
        while (i_ < s_.size()) {
            if (starts("<!--")) skip_to("-->");
            else if (starts("<?")) skip_to("?>");
            else if (starts("<!")) skip_to(">");
            else if (s_[i_] == '<') return;
            else ++i_;
        }
    }
    std::string name() {
        size_t b = i_;
        while (i_ < s_.size()) {
            char c = s_[i_];
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '/' || c == '>' || c == '=') break;
            ++i_;
        }
        if (b == i_) throw err("expected a name");
        return s_.substr(b, i_ - b);
    }
    static std::string unescape(const std::string& v) {
        std::string o;
        o.reserve(v.size());
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] != '&') { o += v[k]; continue; }
            static const char* ent[5][2] = {{"&lt;", "<"}, {"&gt;", ">"}, {"&amp;", "&"}, {"&quot;", "\""}, {"&apos;", "'"}};
            bool hit = false;
            for (auto& e : ent) {
                size_t L = std::strlen(e[0]);
                if (v.compare(k, L, e[0]) == 0) { o += e[1]; k += L - 1; hit = true; break; }
            }
            if (!hit) o += '&';
        }
        return o;
    }
    std::unique_ptr<XNode> element() {
        ++i_;  // '<'
        auto n = std::make_unique<XNode>();
        n->tag = name();
        while (true) {
            ws();
            if (i_ >= s_.size()) throw err("unterminated tag");
            if (starts("/>")) { i_ += 2; return n; }
            if (s_[i_] == '>') { ++i_; break; }
            std::string an = name();
            ws();
            if (i_ >= s_.size() || s_[i_] != '=') throw err("expected '='");
            ++i_;
            ws();
            char q = s_[i_];
            if (q != '"' && q != '\'') throw err("expected quoted attribute value");
            size_t e = s_.find(q, i_ + 1);
            if (e == std::string::npos) throw err("unterminated attribute value");
            n->attrs.emplace_back(an, unescape(s_.substr(i_ + 1, e - i_ - 1)));
            i_ = e + 1;
        }
        while (true) {  // children
            skip_misc();
            if (i_ >= s_.size()) throw err("missing closing tag");
            if (starts("</")) {
                i_ += 2;
                std::string cn = name();
                if (cn != n->tag) throw err("mismatched closing tag");
                ws();
                if (s_[i_] != '>') throw err("expected '>'");
                ++i_;
                return n;
            }
            n->kids.push_back(element());
        }
    }
};

}  // namespace sspp
