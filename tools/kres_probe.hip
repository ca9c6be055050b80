// Compile-only probe of the register-resident 256^2 kernels' resources (VGPRs, spills, LDS): each kernel is
// instantiated by a launch that never runs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGD_KERNELS_ONLY -Rpass-analysis=kernel-resource-usage \
//         -o /tmp/kres tools/kres_probe.hip 2>&1 | python3 tools/resource_report.py "k_"
#include "../galaxy-deconv_amd/csrc/gd_engine.hip"
int main(int argc, char**) {
    if (argc > 1000) {  // never true: instantiation only
        gd::Args a{};
        hipLaunchKernelGGL((gd::k_gal_reg<256, false>), dim3(1), dim3(512), 0, 0, a);
        hipLaunchKernelGGL((gd::k_gal_reg<256, true>), dim3(1), dim3(512), 0, 0, a);
        hipLaunchKernelGGL((gd::k_gal_reg_init<256, false>), dim3(1), dim3(512), 0, 0, a);
        hipLaunchKernelGGL((gd::k_gal_reg_init<256, true>), dim3(1), dim3(512), 0, 0, a);
        hipLaunchKernelGGL((gd::k_pois_b<256>), dim3(1), dim3(512), 0, 0, a, 0);
        hipLaunchKernelGGL((gd::k_rl_reg<256>), dim3(1), dim3(512), 0, 0, a, 1);
    }
    return 0;
}
