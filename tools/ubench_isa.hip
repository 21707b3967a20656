// ubench_isa.hip — issue rate of single VALU instructions on gfx950 with
// explicitly placed registers (measurement tool, not product code).
//
// Each probe issues 8 independent instructions per step (destinations
// v8..v15, never read; sources from v16..v47, never written), 16 steps per
// loop iteration, at 8 waves per SIMD. VGPR bank = register index mod 4, so
// "same bank" / "diff bank" variants show whether an instruction's rate
// depends on reading two operands from one bank. Also times the BLAKE3
// compression loop with alternative rotate implementations.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define R8(I0, I1, I2, I3, I4, I5, I6, I7) I0 "\n" I1 "\n" I2 "\n" I3 "\n" I4 "\n" I5 "\n" I6 "\n" I7 "\n"
#define CLOB                                                                                                  \
  "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", \
      "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38",  \
      "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47"

template <int OP>
__global__ void __launch_bounds__(256) k_probe(uint32_t* out, int iters) {
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      // v16.. : bank 0 = v16,v20,v24..; bank 1 = v17,v21..; bank 2 = v18..; bank 3 = v19..
      if (OP == 0)
        asm volatile(R8("v_add_u32 v8, v16, v17", "v_add_u32 v9, v20, v21", "v_add_u32 v10, v24, v25",
                        "v_add_u32 v11, v28, v29", "v_add_u32 v12, v32, v33", "v_add_u32 v13, v36, v37",
                        "v_add_u32 v14, v40, v41", "v_add_u32 v15, v44, v45") ::: CLOB);
      if (OP == 1)  // alignbit, the same register twice (rotate)
        asm volatile(R8("v_alignbit_b32 v8, v16, v16, 7", "v_alignbit_b32 v9, v17, v17, 7",
                        "v_alignbit_b32 v10, v18, v18, 7", "v_alignbit_b32 v11, v19, v19, 7",
                        "v_alignbit_b32 v12, v20, v20, 7", "v_alignbit_b32 v13, v21, v21, 7",
                        "v_alignbit_b32 v14, v22, v22, 7", "v_alignbit_b32 v15, v23, v23, 7") ::: CLOB);
      if (OP == 2)  // alignbit, two registers in different banks
        asm volatile(R8("v_alignbit_b32 v8, v16, v17, 7", "v_alignbit_b32 v9, v18, v19, 7",
                        "v_alignbit_b32 v10, v20, v21, 7", "v_alignbit_b32 v11, v22, v23, 7",
                        "v_alignbit_b32 v12, v24, v25, 7", "v_alignbit_b32 v13, v26, v27, 7",
                        "v_alignbit_b32 v14, v28, v29, 7", "v_alignbit_b32 v15, v30, v31, 7") ::: CLOB);
      if (OP == 3)  // alignbit, two registers in the same bank
        asm volatile(R8("v_alignbit_b32 v8, v16, v20, 7", "v_alignbit_b32 v9, v17, v21, 7",
                        "v_alignbit_b32 v10, v18, v22, 7", "v_alignbit_b32 v11, v19, v23, 7",
                        "v_alignbit_b32 v12, v24, v28, 7", "v_alignbit_b32 v13, v25, v29, 7",
                        "v_alignbit_b32 v14, v26, v30, 7", "v_alignbit_b32 v15, v27, v31, 7") ::: CLOB);
      if (OP == 4)  // add3, three banks
        asm volatile(R8("v_add3_u32 v8, v16, v17, v18", "v_add3_u32 v9, v20, v21, v22",
                        "v_add3_u32 v10, v24, v25, v26", "v_add3_u32 v11, v28, v29, v30",
                        "v_add3_u32 v12, v32, v33, v34", "v_add3_u32 v13, v36, v37, v38",
                        "v_add3_u32 v14, v40, v41, v42", "v_add3_u32 v15, v44, v45, v46") ::: CLOB);
      if (OP == 5)  // bitop3 (xor3), three banks
        asm volatile(R8("v_bitop3_b32 v8, v16, v17, v18 bitop3:0x96", "v_bitop3_b32 v9, v20, v21, v22 bitop3:0x96",
                        "v_bitop3_b32 v10, v24, v25, v26 bitop3:0x96", "v_bitop3_b32 v11, v28, v29, v30 bitop3:0x96",
                        "v_bitop3_b32 v12, v32, v33, v34 bitop3:0x96", "v_bitop3_b32 v13, v36, v37, v38 bitop3:0x96",
                        "v_bitop3_b32 v14, v40, v41, v42 bitop3:0x96",
                        "v_bitop3_b32 v15, v44, v45, v46 bitop3:0x96") ::: CLOB);
      if (OP == 6)  // rotr16 as a packed 16-bit add with swapped halves
        asm volatile(R8("v_pk_add_u16 v8, v16, 0 op_sel:[1,0] op_sel_hi:[0,0]",
                        "v_pk_add_u16 v9, v17, 0 op_sel:[1,0] op_sel_hi:[0,0]",
                        "v_pk_add_u16 v10, v18, 0 op_sel:[1,0] op_sel_hi:[0,0]",
                        "v_pk_add_u16 v11, v19, 0 op_sel:[1,0] op_sel_hi:[0,0]",
                        "v_pk_add_u16 v12, v20, 0 op_sel:[1,0] op_sel_hi:[0,0]",
                        "v_pk_add_u16 v13, v21, 0 op_sel:[1,0] op_sel_hi:[0,0]",
                        "v_pk_add_u16 v14, v22, 0 op_sel:[1,0] op_sel_hi:[0,0]",
                        "v_pk_add_u16 v15, v23, 0 op_sel:[1,0] op_sel_hi:[0,0]") ::: CLOB);
      if (OP == 7)  // perm
        asm volatile(R8("v_perm_b32 v8, v16, v17, v40", "v_perm_b32 v9, v18, v19, v41",
                        "v_perm_b32 v10, v20, v21, v42", "v_perm_b32 v11, v22, v23, v43",
                        "v_perm_b32 v12, v24, v25, v44", "v_perm_b32 v13, v26, v27, v45",
                        "v_perm_b32 v14, v28, v29, v46", "v_perm_b32 v15, v30, v31, v47") ::: CLOB);
      if (OP == 8)  // add3 with a literal-free SGPR-free form but two same-bank sources
        asm volatile(R8("v_add3_u32 v8, v16, v20, v17", "v_add3_u32 v9, v21, v25, v18",
                        "v_add3_u32 v10, v24, v28, v19", "v_add3_u32 v11, v29, v33, v26",
                        "v_add3_u32 v12, v32, v36, v27", "v_add3_u32 v13, v37, v41, v34",
                        "v_add3_u32 v14, v40, v44, v35", "v_add3_u32 v15, v45, v17, v42") ::: CLOB);
      if (OP == 9)  // VOP3-encoded plain add (e64)
        asm volatile(R8("v_add_u32_e64 v8, v16, v17", "v_add_u32_e64 v9, v20, v21", "v_add_u32_e64 v10, v24, v25",
                        "v_add_u32_e64 v11, v28, v29", "v_add_u32_e64 v12, v32, v33", "v_add_u32_e64 v13, v36, v37",
                        "v_add_u32_e64 v14, v40, v41", "v_add_u32_e64 v15, v44, v45") ::: CLOB);
      if (OP == 10)  // lshl_or
        asm volatile(R8("v_lshl_or_b32 v8, v16, 7, v17", "v_lshl_or_b32 v9, v20, 7, v21",
                        "v_lshl_or_b32 v10, v24, 7, v25", "v_lshl_or_b32 v11, v28, 7, v29",
                        "v_lshl_or_b32 v12, v32, 7, v33", "v_lshl_or_b32 v13, v36, 7, v37",
                        "v_lshl_or_b32 v14, v40, 7, v41", "v_lshl_or_b32 v15, v44, 7, v45") ::: CLOB);
      if (OP == 11)  // xad
        asm volatile(R8("v_xad_u32 v8, v16, v17, v18", "v_xad_u32 v9, v20, v21, v22", "v_xad_u32 v10, v24, v25, v26",
                        "v_xad_u32 v11, v28, v29, v30", "v_xad_u32 v12, v32, v33, v34",
                        "v_xad_u32 v13, v36, v37, v38", "v_xad_u32 v14, v40, v41, v42",
                        "v_xad_u32 v15, v44, v45, v46") ::: CLOB);
      if (OP == 12)  // lshrrev (VOP2)
        asm volatile(R8("v_lshrrev_b32 v8, 7, v16", "v_lshrrev_b32 v9, 7, v17", "v_lshrrev_b32 v10, 7, v18",
                        "v_lshrrev_b32 v11, 7, v19", "v_lshrrev_b32 v12, 7, v20", "v_lshrrev_b32 v13, 7, v21",
                        "v_lshrrev_b32 v14, 7, v22", "v_lshrrev_b32 v15, 7, v23") ::: CLOB);
      if (OP == 13)  // alignbyte (byte rotate), same register twice
        asm volatile(R8("v_alignbyte_b32 v8, v16, v16, 1", "v_alignbyte_b32 v9, v17, v17, 1",
                        "v_alignbyte_b32 v10, v18, v18, 1", "v_alignbyte_b32 v11, v19, v19, 1",
                        "v_alignbyte_b32 v12, v20, v20, 1", "v_alignbyte_b32 v13, v21, v21, 1",
                        "v_alignbyte_b32 v14, v22, v22, 1", "v_alignbyte_b32 v15, v23, v23, 1") ::: CLOB);
      if (OP == 14)  // xor SDWA: hi word <- lo ^ lo (rotr16 half)
        asm volatile(R8("v_xor_b32_sdwa v8, v16, v17 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
                        "v_xor_b32_sdwa v9, v20, v21 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
                        "v_xor_b32_sdwa v10, v24, v25 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
                        "v_xor_b32_sdwa v11, v28, v29 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
                        "v_xor_b32_sdwa v12, v32, v33 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
                        "v_xor_b32_sdwa v13, v36, v37 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
                        "v_xor_b32_sdwa v14, v40, v41 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
                        "v_xor_b32_sdwa v15, v44, v45 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0") ::: CLOB);
      if (OP == 15)  // mixed: 1 alignbit + 1 add (VOP3 next to VOP2)
        asm volatile(R8("v_alignbit_b32 v8, v16, v16, 7", "v_add_u32 v9, v20, v21", "v_alignbit_b32 v10, v18, v18, 7",
                        "v_add_u32 v11, v28, v29", "v_alignbit_b32 v12, v20, v20, 7", "v_add_u32 v13, v36, v37",
                        "v_alignbit_b32 v14, v22, v22, 7", "v_add_u32 v15, v44, v45") ::: CLOB);
      if (OP == 16)  // 4 alignbit then 4 add
        asm volatile(R8("v_alignbit_b32 v8, v16, v16, 7", "v_alignbit_b32 v10, v18, v18, 7",
                        "v_alignbit_b32 v12, v20, v20, 7", "v_alignbit_b32 v14, v22, v22, 7",
                        "v_add_u32 v9, v20, v21", "v_add_u32 v11, v28, v29", "v_add_u32 v13, v36, v37",
                        "v_add_u32 v15, v44, v45") ::: CLOB);
      if (OP == 17)  // 8 alignbit, then (next step) 8 add
      {
        if (r & 1)
          asm volatile(R8("v_add_u32 v8, v16, v17", "v_add_u32 v9, v20, v21", "v_add_u32 v10, v24, v25",
                          "v_add_u32 v11, v28, v29", "v_add_u32 v12, v32, v33", "v_add_u32 v13, v36, v37",
                          "v_add_u32 v14, v40, v41", "v_add_u32 v15, v44, v45") ::: CLOB);
        else
          asm volatile(R8("v_alignbit_b32 v8, v16, v16, 7", "v_alignbit_b32 v9, v17, v17, 7",
                          "v_alignbit_b32 v10, v18, v18, 7", "v_alignbit_b32 v11, v19, v19, 7",
                          "v_alignbit_b32 v12, v20, v20, 7", "v_alignbit_b32 v13, v21, v21, 7",
                          "v_alignbit_b32 v14, v22, v22, 7", "v_alignbit_b32 v15, v23, v23, 7") ::: CLOB);
      }
      if (OP == 18)  // 2 alignbit, 2 add
        asm volatile(R8("v_alignbit_b32 v8, v16, v16, 7", "v_alignbit_b32 v10, v18, v18, 7",
                        "v_add_u32 v9, v20, v21", "v_add_u32 v11, v28, v29",
                        "v_alignbit_b32 v12, v20, v20, 7", "v_alignbit_b32 v14, v22, v22, 7",
                        "v_add_u32 v13, v36, v37", "v_add_u32 v15, v44, v45") ::: CLOB);
      if (OP == 19)  // alignbit + bitop3 interleaved
        asm volatile(R8("v_alignbit_b32 v8, v16, v16, 7", "v_bitop3_b32 v9, v20, v21, v22 bitop3:0x96",
                        "v_alignbit_b32 v10, v18, v18, 7", "v_bitop3_b32 v11, v28, v29, v30 bitop3:0x96",
                        "v_alignbit_b32 v12, v20, v20, 7", "v_bitop3_b32 v13, v36, v37, v38 bitop3:0x96",
                        "v_alignbit_b32 v14, v22, v22, 7", "v_bitop3_b32 v15, v44, v45, v46 bitop3:0x96") ::: CLOB);
    }
  }
  if (threadIdx.x == 0 && iters < 0) out[blockIdx.x] = 1;
}

static const char* kNames[] = {"v_add_u32 (VOP2)",           "v_alignbit x,x (rotate)",   "v_alignbit diff banks",
                               "v_alignbit same bank",       "v_add3_u32 3 banks",        "v_bitop3_b32 3 banks",
                               "v_pk_add_u16 opsel (rot16)", "v_perm_b32",                "v_add3_u32 2 same bank",
                               "v_add_u32_e64 (VOP3 enc)",   "v_lshl_or_b32",             "v_xad_u32",
                               "v_lshrrev_b32 (VOP2)",       "v_alignbyte x,x (rot8)",    "v_xor_b32_sdwa",
                               "alignbit+add interleaved",   "4 alignbit + 4 add",        "8 alignbit | 8 add",
                               "2 alignbit + 2 add",         "alignbit+bitop3 interleaved"};

template <int OP>
float run(int blocks, int iters, uint32_t* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 8);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_probe<OP>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

template <int OP>
void report(int blocks, int iters, uint32_t* out) {
  float ms = run<OP>(blocks, iters, out);
  double ops = (double)blocks * 256 * iters * 16 * 8;
  printf("%-30s %8.3f ms  %6.1f T lane-ops/s\n", kNames[OP], ms, ops / ms / 1e9);
}

int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  uint32_t* out;
  hipMalloc(&out, 1 << 20);
  const int blocks = cus * 8;  // 8 waves per SIMD
  report<0>(blocks, iters, out);
  report<1>(blocks, iters, out);
  report<2>(blocks, iters, out);
  report<3>(blocks, iters, out);
  report<4>(blocks, iters, out);
  report<5>(blocks, iters, out);
  report<6>(blocks, iters, out);
  report<7>(blocks, iters, out);
  report<8>(blocks, iters, out);
  report<9>(blocks, iters, out);
  report<10>(blocks, iters, out);
  report<11>(blocks, iters, out);
  report<12>(blocks, iters, out);
  report<13>(blocks, iters, out);
  report<14>(blocks, iters, out);
  report<15>(blocks, iters, out);
  report<16>(blocks, iters, out);
  report<17>(blocks, iters, out);
  report<18>(blocks, iters, out);
  report<19>(blocks, iters, out);
  // occupancy sweep of the interleaved mix
  for (int w = 1; w <= 8; w *= 2) {
    float ms = run<15>(cus * w, iters, out);
    printf("alignbit+add interleaved, %d waves/SIMD: %.1f T lane-ops/s\n", w, (double)cus * w * 256 * iters * 128 / ms / 1e9);
  }
  return 0;
}
