/* TEST INFRASTRUCTURE ONLY — linked into oracle/_ref/libref_td.so next to the reference's own scalar
 * turbo decoder PHY/CODING/3gpplte_turbo_decoder.c (compiled unmodified).  Not a stand-in for any
 * reference behaviour: PHY/CODING/lte_interleaver_inline.h:29-30 declares the QPP walker's two state
 * words `extern`, and the reference defines them in PHY/CODING/3gpplte.c:42-43 (a TU this library does
 * not build).  They are plain storage: threegpplte_interleaver_reset() (lte_interleaver_inline.h:32-36)
 * zeroes both before every pass that reads them (3gpplte_turbo_decoder.c:978, :995).  Declared with
 * the header's type (unsigned int; 3gpplte.c:42-43 spells it uint32_t), no initialiser. */
unsigned int threegpplte_interleaver_output;
unsigned int threegpplte_interleaver_tmp;
