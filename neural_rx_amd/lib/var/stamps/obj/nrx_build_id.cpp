extern "C" const char* nrx_build_id(void) { return "0b900a55479a3e5a+-DNRX_STAMPS"; }
