/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of dlsim's channel stage (closing
 * dlsim's loop for the BLER curves the reference holds), a plain-C restatement of the reference's
 * code; never linked into the product library.
 *
 *   signal_energy     PHY/TOOLS/signal_energy.c:66-110 (MMX pmaddwd / psrad 4 / paddd sums, the
 *                     16-bit DC lane sums, `temp /= length` and `temp2 /= length * length` with an
 *                     unsigned length).  Pinned to the reference TU compiled here
 *                     (oracle/_ref/libref_tools.so, tests/test_dlsim_cpu.py).
 *   randominit / uniformrandom / gaussdouble
 *                     SIMULATION/TOOLS/rangen_double.c:47-118: multiplicative LCG (a = 1664525,
 *                     mod 2^32, odd seed) behind a 97-entry shuffle table, and the polar Box-Muller
 *                     method caching its second deviate.  (That TU includes PHY/defs.h and is not
 *                     buildable here; restated.)
 *   AWGN              SIMULATION/LTE_PHY/dlsim.c:2852-2866: sigma2_dB = 10 log10(tx_lev)
 *                     + 10 log10(N / (12 NB_RB)) - SNR - pa_dB; per sample the I then the Q
 *                     component, r = (short)(s + sqrt(sigma2 / 2) gaussdouble(0, 1)) (iqim = 0).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oai_oracle.h"

int32_t orc_signal_energy(const int32_t *input, uint32_t length)
{
  uint32_t acc = 0;
  uint16_t dre = 0, dim = 0;
  for (uint32_t i = 0; i < (length >> 1) * 2; i++) {
    int16_t v[2];
    memcpy(v, &input[i], 4);
    const int32_t p = (int32_t)((uint32_t)((int32_t)v[0] * v[0]) + (uint32_t)((int32_t)v[1] * v[1]));
    acc += (uint32_t)(p >> 4);
    dre = (uint16_t)(dre + (uint16_t)v[0]);
    dim = (uint16_t)(dim + (uint16_t)v[1]);
  }
  int32_t temp = (int32_t)acc;
  temp = (int32_t)((uint32_t)temp / length);
  temp = (int32_t)((uint32_t)temp << 4);
  const int32_t r = (int16_t)dre, m = (int16_t)dim;
  int32_t temp2 = (int32_t)((uint32_t)(r * r) + (uint32_t)(m * m));
  temp2 = (int32_t)((uint32_t)temp2 / (length * length));
  temp -= temp2;
  return temp > 0 ? temp : 1;
}

/* rangen_double.c state: seed, iy, ir[98]; gaussdouble's cached deviate */
static uint32_t g_seed, g_iy, g_ir[98];
static int g_iset;
static double g_gset;

void orc_randominit(uint32_t seed_init)
{
  g_seed = seed_init ? seed_init : 1u;                   /* the reference draws a time-based seed for 0 */
  if (g_seed % 2 == 0) g_seed += 1;
  for (int i = 1; i <= 97; i++) {
    g_seed = 1664525u * g_seed;
    g_ir[i] = g_seed;
  }
  g_iy = 1;
  g_iset = 0;
}

double orc_uniformrandom(void)
{
  const int j = (int)(1 + 97.0 * g_iy / 4294967296.0);
  g_iy = g_ir[j];
  g_seed = 1664525u * g_seed;
  g_ir[j] = g_seed;
  return (double)g_iy / 4294967296.0;
}

double orc_gaussdouble(double mean, double variance)
{
  if (g_iset == 0) {
    double v1, v2, r;
    do {
      v1 = 2.0 * orc_uniformrandom() - 1.0;
      v2 = 2.0 * orc_uniformrandom() - 1.0;
      r = v1 * v1 + v2 * v2;
    } while (r >= 1.0);
    const double fac = sqrt(-2.0 * log(r) / r);
    g_gset = v1 * fac;
    g_iset = 1;
    return sqrt(variance) * v2 * fac + mean;
  }
  g_iset = 0;
  return sqrt(variance) * g_gset + mean;
}

double orc_awgn_sigma2(int32_t tx_lev, double offset_db)
{
  return pow(10, (10 * log10((double)tx_lev) + offset_db) / 10);
}

void orc_awgn(const int32_t *tx, int32_t *rx, uint32_t n, double sigma2)
{
  const double s = sqrt(sigma2 / 2);
  for (uint32_t i = 0; i < n; i++) {
    int16_t v[2], o[2];
    memcpy(v, &tx[i], 4);
    /* (short) of the double: truncation through int (the values stay far inside int16 here) */
    o[0] = (int16_t)(int32_t)((double)v[0] + s * orc_gaussdouble(0.0, 1.0));
    o[1] = (int16_t)(int32_t)((double)v[1] + s * orc_gaussdouble(0.0, 1.0));
    memcpy(&rx[i], o, 4);
  }
}
