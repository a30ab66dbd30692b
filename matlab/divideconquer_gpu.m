function Sigmaout = divideconquer_gpu(Y, g, k, BURNIN, MCMC, thin, rho, seed)
% DIVIDECONQUER_GPU  Sigmaout = divideconquer_gpu(Y,g,k,BURNIN,MCMC,thin,rho[,seed])
% Same arguments and output as divideconquer.m:1 (posterior-mean covariance in the
% permuted, standardised coordinates, quirk Q7), with the driver (dc:29-87) and the loop
% (dc:90-197) run by libdcfm through the dcfm_mex gateway (matlab/dcfm_mex.c):
%   dc:31-39  zero-column scan here (nnz), kept columns passed by index;
%   dc:48-59  partition + standardisation on the GPU (set_data_raw);
%   dc:68-87  initial state on the GPU from the library's Philox stream (init_state);
%   dc:90-197 the Gibbs sweep and covariance assembly (run), read back (get_sigma).
% varind = randperm(p) (dc:50) is drawn from MATLAB's stream as in the reference.
if nargin < 8, seed = 0; end
[n, p0] = size(Y);
keepcols = find(arrayfun(@(j) nnz(Y(:, j)), 1:p0) > 0);   % dc:31-38
p = numel(keepcols);
P = p / g; K = k / g;
if P ~= fix(P) || K ~= fix(K)
    error('dcfm:shape', 'P = p/g = %g and K = k/g = %g must be integers (dc:41)', P, K);
end
varind = randperm(p);                                      % dc:50
cfg = struct('n', n, 'P', P, 'g', g, 'K', K, 'rho', rho, 'burnin', BURNIN, 'mcmc', MCMC, ...
             'thin', thin, 'as', 1, 'bs', 0.3, 'df', 3, 'ad1', 2, 'bd1', 1, 'ad2', 2, 'bd2', 1, ...
             'seed', seed);
h = dcfm_mex('create', cfg);
cleanup = onCleanup(@() dcfm_mex('destroy', h));
dcfm_mex('set_data_raw', h, Y, int64(keepcols(varind) - 1));  % dc:48-59 on the device
dcfm_mex('init_state', h);                                     % dc:68-87 on the device
dcfm_mex('run', h, 1, BURNIN + MCMC);                          % dc:90-197
Sigmaout = dcfm_mex('get_sigma', h, p);
end
