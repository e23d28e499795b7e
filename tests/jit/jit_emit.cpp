// Emit the hiprtc source of the tree-specialised kernels (plk_jit.hpp: jit_tree4_source,
// plk_jitm.hpp: jit_treeM4_source) for a small two-fragment program, so that
// tests/test_jit_sources.py can cross-compile it for gfx950 with hipcc on a machine without
// a GPU (the library compiles these sources only at run time, on the device).
//   jit_emit <tree4|treeM> <C> <scale 0|1> [S (treeM: 20 | 4)] > kernel.hip
//   jit_emit tree4q <C> 0 > kernel.hip: one class per workgroup with a quad unit (JitShape::cls)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "plk_jit.hpp"
#include "plk_jitm.hpp"

using namespace plk;

int main(int argc, char** argv) {
  const std::string kind = argc > 1 ? argv[1] : "tree4";
  const int C = argc > 2 ? std::atoi(argv[2]) : 4;
  const bool scale = argc > 3 && std::atoi(argv[3]) != 0;
  const int S = argc > 4 ? std::atoi(argv[4]) : 20;
  // 7 tips (0..6), internal nodes 7..11.  Fragment 0: node 10 = ((t0, t1)8, (t2, t3)9),
  // stored in slot 0.  Fragment 1 (root 11): (t4, t5)7 unstored, t6, slot 0 via branch 10.
  // treeM programs carry unstored cherries as T_CHERRY rows instead.
  std::vector<TInstr> prog;
  auto add = [&](int op, int d, int a, int b) { prog.push_back(TInstr{op, d, a, b}); };
  const bool m = kind == "treeM" || kind == "treeM_deep";
  if (m) {
    add(T_CHERRY, 0, 0, 8);
    add(T_CHERRY, 0, 1, 9);
  } else {
    add(T_DESCEND, 1, 0, 0);
    add(T_TIP, 1, 0, 0);
    add(T_TIP, 1, 1, 1);
    add(T_ASCEND, 1, -1, 8);
    add(T_DESCEND, 1, 0, 0);
    add(T_TIP, 1, 2, 2);
    add(T_TIP, 1, 3, 3);
    add(T_ASCEND, 1, -1, 9);
  }
  add(T_ROOT, 0, 0, 0);
  const int start1 = (int)prog.size();
  if (m) {
    add(T_CHERRY, 0, 2, 7);
  } else {
    add(T_DESCEND, 1, 0, 0);
    add(T_TIP, 1, 4, 4);
    add(T_TIP, 1, 5, 5);
    add(T_ASCEND, 1, -1, 7);
  }
  add(T_TIP, 0, 6, 6);
  add(T_DESCEND, 1, 0, 0);  // a one-child internal level: exercises ASCEND with a store
  add(T_LOAD, 1, 0, 10);
  add(T_ASCEND, 1, 1, 11);
  add(T_ROOT, 0, -1, 1);
  std::vector<int32_t> starts = {0, start1};
  // treeM_deep <height>: one fragment over a balanced subtree of that height (cherries as
  // table rows), i.e. height - 1 register levels below the root -- the register pressure of
  // a real cfg3 fragment (DM 4: height 5)
  if (kind == "tree4q") {
    // one fragment, root 11 = (Q 10 = ((t0, t1)8, (t2, t3)9), (t4, t5)7, t6): a quad, a cherry, a tip
    prog.clear();
    add(T_DESCEND, 1, 0, 0);
    add(T_DESCEND, 2, 0, 0);
    add(T_TIP, 2, 0, 0);
    add(T_TIP, 2, 1, 1);
    add(T_ASCEND, 2, -1, 8);
    add(T_DESCEND, 2, 0, 0);
    add(T_TIP, 2, 2, 2);
    add(T_TIP, 2, 3, 3);
    add(T_ASCEND, 2, -1, 9);
    add(T_ASCEND, 1, -1, 10);
    add(T_DESCEND, 1, 0, 0);
    add(T_TIP, 1, 4, 4);
    add(T_TIP, 1, 5, 5);
    add(T_ASCEND, 1, -1, 7);
    add(T_TIP, 0, 6, 6);
    add(T_ROOT, 0, -1, 1);
    starts = {0};
  }
  if (kind == "treeM_deep") {
    prog.clear();
    const int height = argc > 5 ? std::atoi(argv[5]) : 5;
    int next_cherry = 0, next_node = 1000;
    std::function<void(int, int)> sub = [&](int h, int d) {  // a child of height h at level d
      if (h == 1) {
        add(T_CHERRY, d, next_cherry++, next_node++);
        return;
      }
      add(T_DESCEND, d + 1, 0, 0);
      sub(h - 1, d + 1);
      sub(h - 1, d + 1);
      add(T_ASCEND, d + 1, -1, next_node++);
    };
    sub(height - 1, 0);
    sub(height - 1, 0);
    add(T_ROOT, 0, 0, 1);
    starts = {0};
  }
  std::string src;
  if (m) {
    JitMShape sh;
    sh.S = S;
    sh.C = C;
    sh.U = 16;
    sh.scale = scale;
    if (const char* e = std::getenv("JIT_EMIT_PIPE")) sh.pipe = std::atoi(e);
    if (const char* e = std::getenv("JIT_EMIT_LC")) sh.lc = std::atoi(e);
    src = jit_treeM4_source(prog, starts, sh);
  } else {
    JitShape sh;
    sh.C = C;
    sh.CW = argc > 5 && std::atoi(argv[5]) ? C : 1;
    sh.U = 16;
    sh.scale = scale;
    sh.cls = kind == "tree4q";
    if (sh.cls) sh.U = 4;
    const JitPlan plan = sh.cls ? jit_plan(prog, starts, sh.C, sh.U, 136 * 1024 / 8, false, true, 136 * 1024 / 8)
                                : jit_plan(prog, starts, sh.C, sh.U, 64 * 1024 / 8, scale);
    if (sh.cls) {
      int nq = 0;
      for (const JitUnit& u : plan.units[0]) nq += u.tc >= 0;
      if (nq != 1) {
        std::fprintf(stderr, "expected one quad unit, got %d\n", nq);
        return 1;
      }
    }
    sh.NT = plan.NU;
    sh.TD = plan.tab_doubles;
    sh.QT = plan.quad_tmp;
    sh.soa = std::getenv("JIT_EMIT_SOA") != nullptr;
    // JIT_EMIT_DC=<words>: direct codes (one class per workgroup; or every class in the wave, with
    // the given 16-byte words per pattern)
    sh.dc = (sh.cls || sh.CW > 1) && std::getenv("JIT_EMIT_DC") != nullptr;
    if (sh.dc) sh.dcw = std::max(1, std::atoi(std::getenv("JIT_EMIT_DC")));
    sh.G = 1;
    sh.PW = 1;
    sh.L = sh.CW > 1 ? 2 : 3;
    sh.ppipe = true;
    src = jit_tree4_source(plan, sh);
  }
  std::fwrite(src.data(), 1, src.size(), stdout);
  return 0;
}
