// mc_tables.h - marching-cubes case tables, decoded at compile time (constexpr) so the gfx950 kernel
// (__constant__) and the CPU oracle share one definition. edgeTable is derived from the cube's edge
// topology; the triangulation is Paul Bourke's table (mc_tables_data.h), the one the reference
// carries in Source/DepthSensing/Tables.h. tests/test_mc.py checks that the two agree.
#pragma once
#include <stdint.h>

#include "mc_tables_data.h"  // kMcTriCases

namespace bf {

// Cube corners in the order of extractIsoSurfaceAtPosition's cubeindex bits
// (MarchingCubesSDFUtil.h:144-152): 0 p010, 1 p110, 2 p100, 3 p000, 4 p011, 5 p111, 6 p101, 7 p001.
// Edge e joins corners kMcEdgeA[e] -> kMcEdgeB[e], the (p1, p2) order of its vertexInterp call (:181-192).
constexpr uint8_t kMcEdgeA[12] = {0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 2, 3};
constexpr uint8_t kMcEdgeB[12] = {1, 2, 3, 0, 5, 6, 7, 4, 4, 5, 6, 7};

struct McTables {
    uint16_t edges[256];    // edgeTable: edges whose two corners lie on different sides of the iso level
    uint8_t ntri[256];      // triangles per case
    uint8_t tri[256][15];   // triTable without the -1 terminator
};

constexpr int mc_hex(char c) { return c <= '9' ? c - '0' : c - 'a' + 10; }

constexpr McTables make_mc_tables() {
    McTables t{};
    for (int c = 0; c < 256; c++) {
        uint16_t m = 0;
        for (int e = 0; e < 12; e++)
            if (((c >> kMcEdgeA[e]) & 1) != ((c >> kMcEdgeB[e]) & 1)) m = (uint16_t)(m | (1u << e));
        t.edges[c] = m;
        int n = 0;
        for (const char* s = kMcTriCases[c]; *s; s++) t.tri[c][n++] = (uint8_t)mc_hex(*s);
        t.ntri[c] = (uint8_t)(n / 3);
    }
    return t;
}

}  // namespace bf
