// Input tab (datax-pipeline flowDefinition/components/input/inputSettingsContent.jsx): input mode and type, the
// per-type connection fields, batch inputs (batching mode), streaming interval / max rate / event-time column /
// watermark, the input schema editor with "Get schema" (samples the configured input for N seconds:
// inputdata/inferschema), and the normalization snippet (projection).
import { h } from '../common/dom.js';
import { queryApi } from '../common/api.js';
import { TextField, Dropdown, Toggle, Button, StatementBox, ItemList, functionEnabled, userContext } from '../common/components.js';
import * as Models from './models.js';
import * as V from './validation.js';

// the connection field's meaning per input type
const CONNECTION = {
    events: ['Event Hub connection string (Endpoint=sb://...;EntityPath=...)', null],
    iothub: ['IoT Hub Event Hub-compatible connection string', 'Event Hub-compatible name'],
    kafka: ['Bootstrap servers (host:port,...)', 'Topics (comma separated)'],
    kafkaeventhub: ['Event Hubs namespace connection string (Kafka endpoint)', 'Event hubs / topics (comma separated)'],
    socket: ['Listen address (host:port)', null],
    file: ['Folder or glob of JSON-lines files', null],
    local: [null, null]
};

export function interactiveQueryObject(flow, seconds) {
    const p = flow.input.properties;
    return {
        name: flow.name,
        displayName: flow.displayName,
        userName: userContext.user.name || '',
        inputType: flow.input.type,
        inputMode: flow.input.mode,
        eventhubConnectionString: p.inputEventhubConnection,
        eventhubNames: p.inputEventhubName,
        inputSubscriptionId: p.inputSubscriptionId || '',
        inputResourceGroup: p.inputResourceGroup || '',
        seconds: seconds,
        inputSchema: p.inputSchemaFile,
        normalizationSnippet: p.normalizationSnippet,
        referenceDatas: flow.referenceData,
        functions: flow.functions,
        batchInputs: flow.batchInputs
    };
}

function batchInputsEditor(flow, ui) {
    const items = flow.batchInputs;
    let sel = Math.min(ui.selected.batchInputs || 0, items.length - 1);
    const b = items[sel];
    return h(
        'div',
        { class: 'cols' },
        ItemList(items, sel, (x, i) => x.properties.path || `input ${i + 1}`, i => { ui.selected.batchInputs = i; ui.update(); },
            () => { items.push(Models.defaultBatchInput()); ui.selected.batchInputs = items.length - 1; ui.touch(); ui.update(); },
            i => { items.splice(i, 1); if (!items.length) items.push(Models.defaultBatchInput()); ui.touch(); ui.update(); },
            { isValid: V.isBatchInputComplete, canDelete: () => items.length > 1 }),
        b
            ? h(
                'div',
                { class: 'grow' },
                Dropdown('Type', Models.inputTypesBatching, b.type, v => { b.type = v; ui.touch(); }),
                TextField('Storage connection string (optional for local paths)', b.properties.connection, v => { b.properties.connection = v; ui.touch(); }),
                TextField('Path template, e.g. wasbs://c@acct.blob.core.windows.net/data/{yyyy/MM/dd}/ or /data/{yyyy/MM/dd}/',
                    b.properties.path, v => { b.properties.path = v; ui.touch(); }),
                Dropdown('Format', Models.formatTypes, b.properties.formatType, v => { b.properties.formatType = v; ui.touch(); }),
                Dropdown('Compression', Models.inputCompressionTypes, b.properties.compressionType, v => { b.properties.compressionType = v; ui.touch(); })
            )
            : null
    );
}

export function InputTab(flow, ui) {
    const input = flow.input;
    const p = input.properties;
    const batching = input.mode === 'batching';
    const types = batching ? Models.inputTypesBatching : Models.inputTypes;
    const conn = CONNECTION[input.type] || [null, null];
    const en = name => !functionEnabled(name);
    const seconds = { v: '5' };
    const status = h('span', { class: 'muted' });
    const schemaBox = TextField('Input schema (Spark StructType JSON)', p.inputSchemaFile, v => { p.inputSchemaFile = v; ui.touch(); }, {
        multiline: true,
        mono: true,
        height: '260px',
        disabled: en('inputSchemaEditorEnabled'),
        validate: v => (V.isValidJson(v) ? null : 'not valid JSON')
    });

    async function getSchema() {
        status.textContent = `sampling the input for ${seconds.v} s...`;
        try {
            const res = await queryApi.inferSchema(interactiveQueryObject(flow, Number(seconds.v) || 5));
            p.inputSchemaFile = typeof res.Schema === 'string' ? res.Schema : JSON.stringify(res.Schema || res, null, 2);
            ui.touch();
            ui.update();
        } catch (e) {
            status.textContent = 'Get schema failed: ' + e.message;
        }
    }

    return h(
        'div',
        null,
        h(
            'div',
            { class: 'row' },
            Dropdown('Mode', Models.inputModes, input.mode, v => {
                input.mode = v;
                input.type = v === 'batching' ? 'blob' : userContext.enableLocalOneBox ? 'local' : 'events';
                p.normalizationSnippet = v === 'batching' ? Models.defaultBatchNormalizationSnippet : Models.defaultNormalizationSnippet;
                ui.touch();
                ui.update();
            }, { disabled: en('inputModeDropdownEnabled') }),
            Dropdown('Type', types, input.type, v => { input.type = v; ui.touch(); ui.update(); }, { disabled: en('inputTypeDropdownEnabled') })
        ),
        batching ? batchInputsEditor(flow, ui) : null,
        !batching && conn[0]
            ? TextField(conn[0], p.inputEventhubConnection, v => { p.inputEventhubConnection = v; ui.touch(); }, {
                disabled: en('inputEventHubConnectionStringEnabled'),
                type: input.type === 'events' || input.type === 'iothub' || input.type === 'kafkaeventhub' ? 'password' : null
            })
            : null,
        !batching && conn[1]
            ? TextField(conn[1], p.inputEventhubName, v => { p.inputEventhubName = v; ui.touch(); }, { disabled: en('inputEventHubEnabled') })
            : null,
        !batching
            ? h(
                'div',
                { class: 'row' },
                TextField('Batch interval (seconds)', p.windowDuration, v => { p.windowDuration = v; ui.touch(); }, {
                    disabled: en('inputWindowDurationTextboxEnabled'),
                    validate: v => (V.isValidNumberAboveZero(v) ? null : 'a number above 0')
                }),
                TextField(input.type === 'local' ? 'Events per batch' : 'Max events per partition per batch', p.maxRate, v => { p.maxRate = v; ui.touch(); }, {
                    disabled: en('inputMaxRateTextboxEnabled'),
                    validate: v => (V.isValidNumberAboveZero(v) ? null : 'a number above 0')
                })
            )
            : null,
        h(
            'div',
            { class: 'row' },
            TextField('Event-time column (for windows; empty = arrival time)', p.timestampColumn, v => { p.timestampColumn = v; ui.touch(); }, {
                disabled: en('inputTimestampColumnEnabled')
            }),
            TextField('Watermark', p.watermarkValue, v => { p.watermarkValue = v; ui.touch(); }, {
                disabled: en('inputWatermarkEnabled'),
                validate: v => (V.isValidNumberAboveOrEqualZero(v) ? null : 'a number ≥ 0')
            }),
            Dropdown('unit', Models.watermarkUnits, p.watermarkUnit, v => { p.watermarkUnit = v; ui.touch(); }, { disabled: en('inputWatermarkEnabled') })
        ),
        h(
            'div',
            { class: 'row' },
            Button('Get schema', getSchema, { disabled: en('getInputSchemaButtonEnabled') }),
            h('span', null, 'sample for'),
            h('input', { value: seconds.v, size: 3, oninput: e => (seconds.v = e.target.value) }),
            h('span', null, 'seconds'),
            status
        ),
        schemaBox,
        Toggle('Edit the normalization snippet', !!p.showNormalizationSnippet, v => { p.showNormalizationSnippet = v; ui.update(); }),
        p.showNormalizationSnippet
            ? TextField('Normalization snippet (one projection expression per line over Raw / Properties / SystemProperties)',
                p.normalizationSnippet, v => { p.normalizationSnippet = v; ui.touch(); }, {
                    multiline: true, mono: true, disabled: en('inputNormalizationEditorEnabled')
                })
            : null,
        StatementBox('i', 'Events are parsed from JSON into columns on the GPU by the schema above; fields it omits are dropped.')
    );
}
