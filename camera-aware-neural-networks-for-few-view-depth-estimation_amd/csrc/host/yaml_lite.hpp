// Minimal YAML subset reader for the training configs (yaml-cpp is absent on this image):
// block mappings by indentation, scalars (plain / single- / double-quoted), flow lists [a, b],
// block lists ("- item"), '#' comments.  That is everything configs/train_config*.yaml use.
// Interface mirrors the yaml-cpp calls of train_main.cpp:60-167: node["key"], node.as<T>(default).
#pragma once
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace yaml_lite {

struct Node {
    enum Kind { Null, Scalar, Map, List } kind = Null;
    std::string scalar;
    std::vector<std::pair<std::string, std::shared_ptr<Node>>> map;
    std::vector<std::shared_ptr<Node>> list;

    explicit operator bool() const { return kind != Null; }
    const Node& operator[](const std::string& k) const {
        static const Node null;
        if (kind != Map) return null;
        for (auto& kv : map)
            if (kv.first == k) return *kv.second;
        return null;
    }
    const Node& operator[](size_t i) const {
        static const Node null;
        return kind == List && i < list.size() ? *list[i] : null;
    }
    size_t size() const { return kind == List ? list.size() : kind == Map ? map.size() : 0; }

    template <class T>
    T as(const T& def) const;
    template <class T>
    T as() const {
        if (kind == Null) throw std::runtime_error("yaml: missing value");
        return as<T>(T());
    }
};

inline std::string trim(const std::string& s) {
    size_t a = s.find_first_not_of(" \t\r"), b = s.find_last_not_of(" \t\r");
    return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}
inline std::string strip_comment(const std::string& s) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == '\'' && !dq) sq = !sq;
        else if (s[i] == '"' && !sq) dq = !dq;
        else if (s[i] == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
    }
    return s;
}
inline std::string unquote(std::string v) {
    v = trim(v);
    if (v.size() >= 2 && ((v.front() == '"' && v.back() == '"') || (v.front() == '\'' && v.back() == '\'')))
        return v.substr(1, v.size() - 2);
    return v;
}
inline std::shared_ptr<Node> scalar_or_flow(const std::string& raw) {
    auto n = std::make_shared<Node>();
    std::string v = trim(raw);
    if (v.empty() || v == "~" || v == "null") return n;
    if (v.front() == '[' && v.back() == ']') {
        n->kind = Node::List;
        std::string body = v.substr(1, v.size() - 2), cur;
        bool sq = false, dq = false;
        for (char c : body) {
            if (c == '\'' && !dq) sq = !sq;
            if (c == '"' && !sq) dq = !dq;
            if (c == ',' && !sq && !dq) {
                if (!trim(cur).empty()) n->list.push_back(scalar_or_flow(cur));
                cur.clear();
            } else {
                cur += c;
            }
        }
        if (!trim(cur).empty()) n->list.push_back(scalar_or_flow(cur));
        return n;
    }
    n->kind = Node::Scalar;
    n->scalar = unquote(v);
    return n;
}

struct Line {
    int indent;
    std::string text;
};

inline bool is_item(const Line& ln) { return ln.text.rfind("- ", 0) == 0 || ln.text == "-"; }

// list_only: a block sequence written at its key's own indentation ("key:\n- a\n- b", the form
// yaml.safe_dump emits) ends at the first line of that indentation that is not an item
inline std::shared_ptr<Node> parse_block(const std::vector<Line>& L, size_t& i, int indent, bool list_only = false) {
    auto node = std::make_shared<Node>();
    while (i < L.size() && L[i].indent >= indent) {
        const Line& ln = L[i];
        if (list_only && ln.indent == indent && !is_item(ln)) break;
        if (ln.indent > indent && node->kind == Node::Null) indent = ln.indent;
        if (ln.indent != indent) throw std::runtime_error("yaml: bad indentation near '" + ln.text + "'");
        if (is_item(ln)) {
            node->kind = Node::List;
            std::string item = ln.text.size() > 1 ? trim(ln.text.substr(2)) : "";
            ++i;
            if (item.empty()) node->list.push_back(parse_block(L, i, indent + 1));
            else node->list.push_back(scalar_or_flow(item));
            continue;
        }
        size_t c = ln.text.find(':');
        if (c == std::string::npos) throw std::runtime_error("yaml: expected 'key: value' near '" + ln.text + "'");
        node->kind = Node::Map;
        std::string key = unquote(ln.text.substr(0, c));
        std::string rest = trim(ln.text.substr(c + 1));
        ++i;
        if (rest.empty()) {
            if (i < L.size() && L[i].indent > indent) node->map.push_back({key, parse_block(L, i, L[i].indent)});
            else if (i < L.size() && L[i].indent == indent && is_item(L[i]))
                node->map.push_back({key, parse_block(L, i, indent, true)});
            else node->map.push_back({key, std::make_shared<Node>()});
        } else {
            node->map.push_back({key, scalar_or_flow(rest)});
        }
    }
    return node;
}

// "key: ..." (a colon outside quotes followed by a blank or the end of the line)
inline bool is_mapping_entry(const std::string& t) {
    if (t.empty() || t.front() == '[') return false;
    bool sq = false, dq = false;
    for (size_t i = 0; i < t.size(); ++i) {
        if (t[i] == '\'' && !dq) sq = !sq;
        else if (t[i] == '"' && !sq) dq = !dq;
        else if (t[i] == ':' && !sq && !dq && (i + 1 == t.size() || t[i + 1] == ' ')) return true;
    }
    return false;
}

inline Node parse(const std::string& text) {
    std::vector<Line> L;
    std::istringstream in(text);
    std::string s;
    while (std::getline(in, s)) {
        s = strip_comment(s);
        if (trim(s).empty() || trim(s) == "---") continue;
        int ind = 0;
        while (ind < (int)s.size() && s[ind] == ' ') ++ind;
        std::string t = trim(s);
        // "- key: v" opens a mapping inside a list item: split it into "-" and "key: v" two columns in
        while (t.rfind("- ", 0) == 0 && is_mapping_entry(trim(t.substr(2)))) {
            L.push_back({ind, "-"});
            ind += 2;
            t = trim(t.substr(2));
        }
        L.push_back({ind, t});
    }
    size_t i = 0;
    if (L.empty()) return Node();
    return *parse_block(L, i, L[0].indent);
}

inline Node load_file(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("Cannot open config file: " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse(ss.str());
}

template <>
inline std::string Node::as<std::string>(const std::string& def) const {
    return kind == Scalar ? scalar : def;
}
template <>
inline float Node::as<float>(const float& def) const {
    return kind == Scalar ? std::strtof(scalar.c_str(), nullptr) : def;
}
template <>
inline double Node::as<double>(const double& def) const {
    return kind == Scalar ? std::strtod(scalar.c_str(), nullptr) : def;
}
template <>
inline int Node::as<int>(const int& def) const {
    return kind == Scalar ? (int)std::strtol(scalar.c_str(), nullptr, 10) : def;
}
template <>
inline bool Node::as<bool>(const bool& def) const {
    if (kind != Scalar) return def;
    return scalar == "true" || scalar == "True" || scalar == "yes" || scalar == "1" || scalar == "on";
}
template <>
inline std::vector<float> Node::as<std::vector<float>>(const std::vector<float>& def) const {
    if (kind != List) return def;
    std::vector<float> v;
    for (auto& n : list) v.push_back(n->as<float>(0.f));
    return v;
}
template <>
inline std::vector<std::string> Node::as<std::vector<std::string>>(const std::vector<std::string>& def) const {
    if (kind != List) return def;
    std::vector<std::string> v;
    for (auto& n : list) v.push_back(n->as<std::string>(""));
    return v;
}

}  // namespace yaml_lite
