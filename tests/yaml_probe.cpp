// test helper: dump a YAML file parsed by yaml_lite as flattened "path=value" lines
#include <iostream>
#include "../camera-aware-neural-networks-for-few-view-depth-estimation_amd/csrc/host/yaml_lite.hpp"
void dump(const yaml_lite::Node& n, const std::string& path) {
    if (n.kind == yaml_lite::Node::Scalar) std::cout << path << "=" << n.scalar << "\n";
    else if (n.kind == yaml_lite::Node::Map) for (auto& kv : n.map) dump(*kv.second, path.empty() ? kv.first : path + "." + kv.first);
    else if (n.kind == yaml_lite::Node::List) for (size_t i = 0; i < n.list.size(); ++i) dump(*n.list[i], path + "[" + std::to_string(i) + "]");
    else std::cout << path << "=~\n";
}
int main(int argc, char** argv) { dump(yaml_lite::load_file(argv[1]), ""); return 0; }
