// K9 per-row LTV / churn / segment logic (ltv.go:113-382): ONE definition for the device (the
// standalone K9 kernel ltv.hip and the fused LTV MLP kernel's epilogue mlp_fused.hip, through
// csrc/kernels/ltv.h) and the host runtime (the CPU LTV device of the native account-RPC core,
// csrc/runtime/acct_devices.cpp). float64 arithmetic like the Go code. Input row =
// golden.ltv.PLAYER_COLUMNS (25 f32); output row = [ltv, churn, survival days, confidence,
// segment id, next-best-action id]. The includer defines IGP_LTV_FN (the function qualifiers).
#pragma once
#ifndef IGP_LTV_FN
#error "define IGP_LTV_FN before including ltv_logic.h"
#endif

namespace igp {

enum { P_DSR = 0, P_DSLD, P_DSLB, P_TAD, P_SPW, P_ASD, P_TDEP, P_TWD, P_NET, P_ADA, P_DFREQ, P_LDEP,
       P_TBETS, P_TWINS, P_BETC, P_WINR, P_ABS, P_GAMES, P_BCLAIM, P_BWAGER, P_BCONV, P_PUSH, P_EMAIL,
       P_VIP, P_TICKETS, P_NCOLS };

IGP_LTV_FN double ltv_engagement(const float* p) {
  double s = 0.0;
  const double dslb = (int)p[P_DSLB];
  if (dslb < 3) s += 0.3; else if (dslb < 7) s += 0.2; else if (dslb < 14) s += 0.1;
  const double spw = p[P_SPW];
  if (spw >= 5) s += 0.2; else if (spw >= 3) s += 0.15; else if (spw >= 1) s += 0.1;
  const double df = p[P_DFREQ];
  if (df >= 4) s += 0.2; else if (df >= 2) s += 0.15; else if (df >= 1) s += 0.1;
  if (p[P_PUSH] != 0.f) s += 0.1;
  if (p[P_EMAIL] != 0.f) s += 0.1;
  if (p[P_VIP] != 0.f) s += 0.1;
  return s < 1.0 ? s : 1.0;
}

// p: the player's profile row; ml: the learned LTV (nullable -> the ltv.go formula); o: 6 floats
IGP_LTV_FN void ltv_row(const float* p, const float* ml, float* o) {
  const int dsr = (int)p[P_DSR], dsld = (int)p[P_DSLD], dslb = (int)p[P_DSLB];
  const double spw = p[P_SPW], net = p[P_NET], df = p[P_DFREQ];
  // churn (ltv.go:228-262)
  double churn = 0.0;
  if (dslb > 30) churn += 0.5; else if (dslb > 14) churn += 0.3; else if (dslb > 7) churn += 0.15;
  if (spw < 1 && dsr > 30) churn += 0.2;
  if (dsld > 30) churn += 0.2;
  if ((int)p[P_TICKETS] > 3) churn += 0.1;
  if ((double)p[P_TWD] > (double)p[P_TDEP]) churn += 0.1;
  churn = churn < 1.0 ? churn : 1.0;
  const double eng = ltv_engagement(p);
  // ltv (ltv.go:155-178) or the learned model
  double ltv;
  if (ml) {
    ltv = (double)*ml;
  } else if (dsr < 30) {
    ltv = net / (double)(dsr > 1 ? dsr : 1) * 30 * 12;
  } else {
    ltv = net + net / (double)dsr * 30 * (12.0 * eng);
  }
  const double adj = ltv * (1 - churn * 0.5);
  int seg;
  if (churn > 0.7) seg = 5;
  else if (adj >= 10000) seg = 1;
  else if (adj >= 1000) seg = 2;
  else if (adj >= 100) seg = 3;
  else seg = 4;
  double surv = 90.0 * (1.0 + eng) * (1.0 - churn);
  const int survival = (int)(surv > 0 ? surv : 0);
  // confidence (ltv.go:346-382)
  double c = 0.0;
  if (dsr > 90) c += 0.3; else if (dsr > 30) c += 0.2; else c += 0.1;
  const int betc = (int)p[P_BETC];
  if (betc > 100) c += 0.3; else if (betc > 20) c += 0.2; else c += 0.1;
  if (df > 2) c += 0.2; else if (df > 0) c += 0.1;
  if (dslb < 7) c += 0.2; else if (dslb < 30) c += 0.1;
  c = c < 1.0 ? c : 1.0;
  // next best action (ltv.go:300-343); ids = golden.ltv.NBA_CODES
  int nba = 0;
  switch (seg) {
    case 5: nba = net > 0 ? 1 : 2; break;
    case 1: nba = dsld > 7 ? 3 : 4; break;
    case 2: nba = p[P_VIP] == 0.f ? 5 : (churn > 0.3 ? 6 : 7); break;
    case 3: nba = (int)p[P_BCLAIM] < 3 ? 8 : ((int)p[P_GAMES] < 5 ? 9 : 10); break;
    case 4: nba = dsr < 7 ? 11 : ((double)p[P_BCONV] > 0.8 ? 0 : 12); break;
  }
  o[0] = (float)adj;
  o[1] = (float)churn;
  o[2] = (float)survival;
  o[3] = (float)c;
  o[4] = (float)seg;
  o[5] = (float)nba;
}

}  // namespace igp
