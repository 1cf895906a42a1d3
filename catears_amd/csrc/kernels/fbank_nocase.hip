// fbank_nocase.hip -- experiments library only, timing only (wrong results):
// the exact fbank kernel with phase A's lane-dependent twiddle cases removed
// (every lane takes the table path; fbank8_ops.h FB8_NOCASE).  It bounds what
// a wave-uniform residue mapping of phase A could save;
// selected by CATEARS_FB_NOCASE=1 for the exact mode.
#ifdef CATEARS_EXPERIMENTS
#define FB8_NOCASE 1
#include "fbank.hip"
#endif
