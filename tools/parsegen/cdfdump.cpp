// cdfdump -- table extraction aid (this container only, never shipped): initialises the
// REFERENCE decoder's default CDFs (decoder/Cdfs.cpp: init_non_coeff_cdfs, and
// init_coeff_cdfs for each of the four quantizer contexts) and prints every CDF leaf as
//   <name> <index...> : <values...>
// The values are the AV1 specification's default CDF tables (libaom's inverted form);
// tools/parsegen/gen_cdf.py turns them into av1dec_amd/csrc/parse/cdf_default.h.
#include "Cdfs.h"
#include <cstdio>
#include <string>
#include <vector>
using namespace YamiAv1;

static void dump(const std::string& name, const std::vector<uint16_t>& v, const std::vector<int>& idx)
{
    printf("%s", name.c_str());
    for (int i : idx) printf(" %d", i);
    printf(" :");
    for (auto x : v) printf(" %u", (unsigned)x);
    printf("\n");
}
template <class T>
static void dump(const std::string& name, const std::vector<T>& v, std::vector<int> idx)
{
    for (size_t i = 0; i < v.size(); i++) {
        idx.push_back((int)i);
        dump(name, v[i], idx);
        idx.pop_back();
    }
}
#define D(m) dump(pre + #m, c.m, {})
int main()
{
    const int qs[4] = {0, 40, 100, 200};  // one base_q_idx per quantizer context (<=20, <=60, <=120, >120)
    for (int qi = 0; qi < 4; qi++) {
        Cdfs c;
        c.init_non_coeff_cdfs();
        c.init_coeff_cdfs(qs[qi]);
        std::string pre = "q" + std::to_string(qi) + ".";
        D(txb_skip_cdf); D(eob_extra_cdf); D(dc_sign_cdf); D(eob_flag_cdf16); D(eob_flag_cdf32); D(eob_flag_cdf64);
        D(eob_flag_cdf128); D(eob_flag_cdf256); D(eob_flag_cdf512); D(eob_flag_cdf1024); D(coeff_base_eob_cdf);
        D(coeff_base_cdf); D(coeff_br_cdf);
        if (qi) continue;
        pre = "";
        D(newmv_cdf); D(zeromv_cdf); D(refmv_cdf); D(drl_cdf); D(inter_compound_mode_cdf); D(compound_type_cdf);
        D(wedge_idx_cdf); D(interintra_cdf); D(wedge_interintra_cdf); D(interintra_mode_cdf); D(motion_mode_cdf);
        D(obmc_cdf); D(palette_y_size_cdf); D(palette_uv_size_cdf); D(palette_y_color_index_cdf);
        D(palette_uv_color_index_cdf); D(palette_y_mode_cdf); D(palette_uv_mode_cdf); D(comp_inter_cdf);
        D(single_ref_cdf); D(comp_ref_type_cdf); D(uni_comp_ref_cdf); D(comp_ref_cdf); D(comp_bwdref_cdf);
        D(txfm_partition_cdf); D(compound_index_cdf); D(comp_group_idx_cdf); D(skip_mode_cdfs); D(skip_cdfs);
        D(intra_inter_cdf); D(intrabc_cdf); D(filter_intra_cdfs); D(filter_intra_mode_cdf); D(switchable_restore_cdf);
        D(wiener_restore_cdf); D(sgrproj_restore_cdf); D(y_mode_cdf); D(uv_mode_cdf); D(partition_cdf);
        D(switchable_interp_cdf); D(kf_y_cdf); D(angle_delta_cdf); D(tx_size_cdf); D(delta_q_cdf);
        D(delta_lf_multi_cdf); D(delta_lf_cdf); D(intra_ext_tx_cdf); D(inter_ext_tx_cdf); D(cfl_sign_cdf);
        D(cfl_alpha_cdf);
        for (int k = 0; k < 2; k++) {
            pre = "nmv" + std::to_string(k) + ".";
            D(nmv_context[k].joints_cdf);
            for (int cpt = 0; cpt < 2; cpt++) {
                pre = "nmv" + std::to_string(k) + ".c" + std::to_string(cpt) + ".";
                D(nmv_context[k].comps[cpt].classes_cdf); D(nmv_context[k].comps[cpt].class0_fp_cdf);
                D(nmv_context[k].comps[cpt].fp_cdf); D(nmv_context[k].comps[cpt].sign_cdf);
                D(nmv_context[k].comps[cpt].class0_hp_cdf); D(nmv_context[k].comps[cpt].hp_cdf);
                D(nmv_context[k].comps[cpt].class0_cdf); D(nmv_context[k].comps[cpt].bits_cdf);
            }
        }
    }
}
