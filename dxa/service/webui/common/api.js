// Service API client (datax-common serviceApi.js / nodeServiceApi.js). The reference posts an envelope to the
// node server, which forwards it to the Service Fabric gateway; here the control plane serves the gateway shape
// /api/{application}/{service}/{route} directly and answers with ApiResult {error, message, result}.

export const Constants = {
    serviceApplication: 'DataX.Flow',
    services: {
        flow: 'Flow.ManagementService',
        interactiveQuery: 'Flow.InteractiveQueryService',
        schemaInference: 'Flow.SchemaInferenceService',
        liveData: 'Flow.LiveDataService'
    }
};

export class ApiError extends Error {
    constructor(message, status) {
        super(message);
        this.status = status;
    }
}

const TOKEN_KEY = 'dxa.bearer';

export function getToken() {
    try {
        return window.localStorage.getItem(TOKEN_KEY) || '';
    } catch (e) {
        return '';
    }
}

export function setToken(t) {
    try {
        if (t) window.localStorage.setItem(TOKEN_KEY, t);
        else window.localStorage.removeItem(TOKEN_KEY);
    } catch (e) {
        /* storage disabled */
    }
}

function headers(json) {
    const h = { Accept: 'application/json' };
    if (json) h['Content-Type'] = 'application/json';
    const t = getToken();
    if (t) h.Authorization = 'Bearer ' + t;
    return h;
}

async function readJson(r) {
    const text = await r.text();
    let j;
    try {
        j = text ? JSON.parse(text) : null;
    } catch (e) {
        throw new ApiError(`${r.status}: ${text.slice(0, 200)}`, r.status);
    }
    if (!r.ok) throw new ApiError((j && (j.detail || j.message)) || `HTTP ${r.status}`, r.status);
    return j;
}

// POST a service route; resolves with ApiResult.result, rejects with ApiError(message) when error is set
export async function servicePost(service, route, body) {
    const r = await fetch(`/api/${Constants.serviceApplication}/${service}/${route}`, {
        method: 'POST',
        headers: headers(true),
        body: JSON.stringify(body === undefined ? {} : body)
    });
    const j = await readJson(r);
    if (j && j.error) throw new ApiError(j.message || 'request failed', r.status);
    return j ? j.result : null;
}

export async function serviceGet(service, route, params) {
    const q = params ? '?' + new URLSearchParams(params).toString() : '';
    const r = await fetch(`/api/${Constants.serviceApplication}/${service}/${route}${q}`, { headers: headers(false) });
    const j = await readJson(r);
    if (j && j.error) throw new ApiError(j.message || 'request failed', r.status);
    return j ? j.result : null;
}

// node-side (website server) GET api: /api/<name>
export async function nodeGet(name, params) {
    const q = params ? '?' + new URLSearchParams(params).toString() : '';
    const r = await fetch(`/api/${name}${q}`, { headers: headers(false) });
    return readJson(r);
}

// flow management shortcuts (datax-pipeline flowDefinition/api.js, flowList/api.js, datax-jobs api.js)
const F = Constants.services.flow;
export const flowApi = {
    getAllMin: () => servicePost(F, 'flow/getall/min'),
    get: name => servicePost(F, 'flow/get', { name }),
    save: flow => servicePost(F, 'flow/save', flow),
    generateConfigs: name => servicePost(F, 'flow/generateconfigs', { name }),
    startJobs: name => servicePost(F, 'flow/startjobs', { name }),
    restartJobs: name => servicePost(F, 'flow/restartjobs', { name }),
    stopJobs: name => servicePost(F, 'flow/stopjobs', { name }),
    remove: name => servicePost(F, 'flow/delete', { name }),
    scheduleBatch: name => servicePost(F, 'flow/schedulebatch', { name }),
    codegen: (query, rules, productId) => servicePost(F, 'userqueries/codegen', { query, rules, productId }),
    schema: (query, inputSchema, rules) => servicePost(F, 'userqueries/schema', { query, inputSchema, rules }),
    conditionsSql: (conditions, ruleType, pivots, aggs) =>
        servicePost(F, 'designer/conditions/sql', { conditions, ruleType, pivots, aggs }),
    toConfig: (flow, query) => servicePost(F, 'designer/flow/toconfig', { flow, query })
};

export const jobApi = {
    getAll: () => servicePost(F, 'job/getall'),
    getByNames: names => servicePost(F, 'job/getbynames', names),
    start: name => servicePost(F, 'job/start', { name }),
    stop: name => servicePost(F, 'job/stop', { name }),
    restart: name => servicePost(F, 'job/restart', { name }),
    syncAll: () => servicePost(F, 'job/syncall')
};

const Q = Constants.services.interactiveQuery;
const S = Constants.services.schemaInference;
const L = Constants.services.liveData;
export const queryApi = {
    createKernel: body => servicePost(Q, 'kernel', body),
    refreshKernel: body => servicePost(Q, 'kernel/refresh', body),
    deleteKernel: kernelId => servicePost(Q, 'kernel/delete', { kernelId }),
    deleteKernels: ids => servicePost(Q, 'kernels/delete', ids),
    deleteAllKernels: () => servicePost(Q, 'kernels/deleteall'),
    executeQuery: (kernelId, query) => servicePost(Q, 'kernel/executequery', { kernelId, query }),
    sampleInput: kernelId => servicePost(Q, 'kernel/sampleinputfromquery', { kernelId }),
    inferSchema: body => servicePost(S, 'inputdata/inferschema', body),
    refreshSample: body => servicePost(S, 'inputdata/refreshsample', body),
    refreshSampleAndKernel: body => servicePost(L, 'inputdata/refreshsampleandkernel', body)
};

export async function getMetricsData(name, startMs, endMs) {
    const r = await fetch(`/api/metrics/get?m=${encodeURIComponent(name)}&s=${startMs}&e=${endMs}`, {
        headers: headers(false)
    });
    return readJson(r);
}

export async function getMetricsFreshness(name) {
    const r = await fetch(`/api/metrics/${encodeURIComponent(name)}/freshness`, { headers: headers(false) });
    return readJson(r);
}
