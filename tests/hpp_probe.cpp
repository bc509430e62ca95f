// Compile/link probe of the C++ drop-in classes (include/cad/cad.hpp) — tests/test_abi.py builds it
// against libcad_hip.so on the CPU; run on a GPU it trains one step of each geometry-aware network.
#include <cstdio>

#include "cad/cad.hpp"

int main() {
    using namespace camera_aware_depth;
    cad::Workspace ws{2, 64, 64, 0};
    GeometryAwareNetworkImpl geo(3, 8, 4, 10.f, true, true, ws);          // geometry_aware_network.h:237-278
    LightweightGeometryNetworkImpl lite(3, 8, 4, 10.f, ws);               // :368-383
    CombinedDepthLoss loss(1.0f, 0.1f, 0.001f, 0.01f, ws);
    std::printf("GeometryAwareNetwork %lld, LightweightGeometryNetwork %lld parameters\n",
                (long long)geo.count_parameters(), (long long)lite.count_parameters());
    return 0;
}
