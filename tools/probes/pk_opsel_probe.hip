// Probe: how gfx950 executes v_pk_*_f32 source-select modifiers (op_sel /
// op_sel_hi) and scalar splats the compiler folds into them.  Prints the
// result of each form next to the value the ISA semantics imply.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void probe(float* out, const float* in) {
  if (threadIdx.x != 0) return;
  f2 a = {in[0], in[1]};     // {1, 100}
  f2 b = {in[2], in[3]};     // {10, 20}
  f2 c = {in[4], in[5]};     // {1000, 2000}
  f2 r;
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  out[0] = r.x; out[1] = r.y;                  // expect 11, 21
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[1,0]" : "=v"(r) : "v"(a), "v"(b));
  out[2] = r.x; out[3] = r.y;                  // expect 110, 120
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  out[4] = r.x; out[5] = r.y;                  // expect 1*10+1000 = 1010, 100*10+2000 = 3000
  asm volatile("v_pk_add_f32 %0, %1, 1.0 op_sel_hi:[1,0]" : "=v"(r) : "v"(a));
  out[6] = r.x; out[7] = r.y;                  // expect 2, 101
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  out[8] = r.x; out[9] = r.y;                  // expect 1-10 = -9, 1-20 = -19
  // compiler-generated splat: scalar minus vector
  volatile float xs = in[0];
  const float xq = xs;
  r = xq - b;
  out[10] = r.x; out[11] = r.y;                // expect -9, -19
}

int main() {
  float h_in[6] = {1.f, 100.f, 10.f, 20.f, 1000.f, 2000.f};
  const float expect[12] = {11, 21, 110, 120, 1010, 3000, 2, 101, -9, -19, -9, -19};
  float *d_in, *d_out, h_out[12];
  hipMalloc(&d_in, sizeof h_in);
  hipMalloc(&d_out, sizeof h_out);
  hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_out, d_in);
  hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost);
  const char* names[6] = {"add op_sel_hi:[0,1]", "add op_sel:[1,0]", "fma op_sel_hi:[1,0,1]", "add 1.0 op_sel_hi:[1,0]",
                          "sub op_sel_hi:[0,1] neg", "compiler splat xq - b"};
  int bad = 0;
  for (int i = 0; i < 6; ++i) {
    const bool ok = h_out[2 * i] == expect[2 * i] && h_out[2 * i + 1] == expect[2 * i + 1];
    bad += !ok;
    printf("%-26s got {%g, %g} expect {%g, %g} %s\n", names[i], h_out[2 * i], h_out[2 * i + 1], expect[2 * i],
           expect[2 * i + 1], ok ? "ok" : "MISMATCH");
  }
  hipFree(d_in);
  hipFree(d_out);
  return bad;
}
