// The wavefront kernels of untextured static sphere scenes (scene features 0 / checker: BASELINE configs 2,
// 3 and 4) as their own translation unit, so that csrc/Makefile can compile them with 64-B loop alignment
// (-falign-loops=64; the gfx9 backend aligns no loop header itself): the fused step's walk and the tail gain
// 0.8 % on C2 and 0.7 % on C3 (C4 -0.4 %); the other scene classes gained nothing from the flag (C5 -0.3 %,
// Cornell -0.4 %) and stay in rtw_wavefront.hip without it (profiles/r4_align_loops/).
#define RTW_WF_SPHERES_TU
#include "rtw_wavefront.hip"
