// Dependency levels of the reach program (development tool, build container): the op tape's
// critical path and how many simplifying operators each level holds, i.e. how much the per-job
// engine could gain by running independent operators on different waves of a job's workgroup
// (DESIGN.md section 8). Slot reuse counts as a dependency (an op may not overwrite a slot an
// earlier op still reads).
//   hipcc -x hip --offload-host-only -O1 -std=c++17 -I armour-dev_amd/csrc -o /tmp/tape_levels \
//         tools/tape_levels.cpp armour-dev_amd/csrc/robots.cpp && /tmp/tape_levels
#include <algorithm>
#include <cstdio>
#include <vector>
#include "reach.h"
#include "robots.h"
using namespace armour;
int main() {
    RobotParams rp;
    kinova_gen3(rp);
    ProgramBuilder pb;
    pb.fused = true;
    pb.build(rp);
    const int n = (int)pb.ops.size();
    std::vector<int> level(n, 0), writer(1024, -1), lastread(1024, -1), simpl(n + 1, 0);
    int maxl = 0, nsimp = 0;
    for (int k = 0; k < n; k++) {
        const Op& op = pb.ops[k];
        std::vector<int> rd;
        switch (op.code) {
            case OP_MUL: case OP_ADD: case OP_ADD1D: case OP_CROSS_PP: rd = {op.a, op.b}; break;
            case OP_STACK3: rd = {op.a, op.b, op.c}; break;
            case OP_VIEW: case OP_TRANSPOSE: case OP_CROSS_C: case OP_EMIT_LINK: case OP_EMIT_TORQUE: rd = {op.a}; break;
            default: break;
        }
        int L = 0;
        for (int s : rd)
            if (s >= 0 && writer[s] >= 0) L = std::max(L, level[writer[s]] + 1);
        if (op.o >= 0) {
            if (writer[op.o] >= 0) L = std::max(L, level[writer[op.o]] + 1);
            if (lastread[op.o] >= 0) L = std::max(L, level[lastread[op.o]] + 1);
        }
        level[k] = L;
        for (int s : rd)
            if (s >= 0) lastread[s] = std::max(lastread[s], k);
        if (op.o >= 0) { writer[op.o] = k; lastread[op.o] = -1; }
        maxl = std::max(maxl, L);
        const bool s = op.code == OP_MUL || op.code == OP_ADD || op.code == OP_ADD1D || op.code == OP_CROSS_PP ||
                       op.code == OP_STACK3 || op.code == OP_CROSS_C;
        simpl[L] += s;
        nsimp += s;
    }
    int hist[8] = {0};
    for (int l = 0; l <= maxl; l++) hist[std::min(simpl[l], 7)]++;
    std::printf("ops %d, dependency levels %d, simplifying ops %d\nlevels holding w simplifying ops:", n, maxl + 1, nsimp);
    for (int w = 0; w < 8; w++) std::printf(" w=%d: %d", w, hist[w]);
    std::printf("\n");
    return 0;
}
