/* layout.c -- sizeof / offsetof of the ABI structs, as the C compiler lays them out, for
 * tests/test_host_cpu.py to compare with the C# StructLayout(Sequential) mirrors in
 * host/csharp/RC2DGINative.cs (Config, Prim). */
#include <stddef.h>
#include <stdio.h>

#include "rc2dgi.h"

#define F(S, m) printf("%s.%s %zu %zu\n", #S, #m, offsetof(S, m), sizeof(((S *)0)->m))

int main(void) {
  printf("rc2dgi_config %zu\n", sizeof(rc2dgi_config));
  F(rc2dgi_config, screen_width);
  F(rc2dgi_config, screen_height);
  F(rc2dgi_config, cascade_count);
  F(rc2dgi_config, render_scale);
  F(rc2dgi_config, ray_range);
  F(rc2dgi_config, storage);
  F(rc2dgi_config, device);
  F(rc2dgi_config, flags);
  F(rc2dgi_config, reserved);
  printf("rc2dgi_prim %zu\n", sizeof(rc2dgi_prim));
  F(rc2dgi_prim, kind);
  F(rc2dgi_prim, x);
  F(rc2dgi_prim, y);
  F(rc2dgi_prim, w);
  F(rc2dgi_prim, h);
  F(rc2dgi_prim, r);
  F(rc2dgi_prim, g);
  F(rc2dgi_prim, b);
  F(rc2dgi_prim, a);
  return 0;
}
