extern "C" const char* rtw_build_id(void) { return "0a9c00991c279de7"; }
